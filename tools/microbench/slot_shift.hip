// store_new_state!'s in-place history shift (slot 3 <- 2 <- 1) of two 4096^2 F64
// (M+2, P+2, 2, 3) arrays: variants of the copy, timed with HIP events.
//   hipcc -O3 --offload-arch=gfx950 slot_shift.hip -o slot_shift && ./slot_shift
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                      \
            return 1;                                                               \
        }                                                                           \
    } while (0)

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store(uint4 v, uint4 *p) {
    u4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u4v *>(p));
}

struct A {
    uint4 *b[2];
    long n;
};

// grid-stride, one vector per iteration
__global__ __launch_bounds__(256) void k_stride(A a) {
    uint4 *b = a.b[blockIdx.y];
    const long n = a.n, st = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += st) {
        const uint4 s1 = b[i], s2 = b[n + i];
        b[n + i] = s1;
        b[2 * n + i] = s2;
    }
}

// V vectors per thread, all loads first
template <int V>
__global__ __launch_bounds__(256) void k_batch(A a) {
    uint4 *b = a.b[blockIdx.y];
    const long n = a.n, i0 = (long)blockIdx.x * (256 * V) + threadIdx.x;
    uint4 s1[V], s2[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const long i = i0 + u * 256;
        if (i < n) {
            s1[u] = b[i];
            s2[u] = b[n + i];
        }
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const long i = i0 + u * 256;
        if (i < n) {
            b[n + i] = s1[u];
            b[2 * n + i] = s2[u];
        }
    }
}

// nontemporal stores
template <int V>
__global__ __launch_bounds__(256) void k_batch_nt(A a) {
    uint4 *b = a.b[blockIdx.y];
    const long n = a.n, i0 = (long)blockIdx.x * (256 * V) + threadIdx.x;
    uint4 s1[V], s2[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const long i = i0 + u * 256;
        if (i < n) {
            s1[u] = b[i];
            s2[u] = b[n + i];
        }
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const long i = i0 + u * 256;
        if (i < n) {
            nt_store(s1[u], b + n + i);
            nt_store(s2[u], b + 2 * n + i);
        }
    }
}

// plain copy (not in place): reference rate of a float4 copy of the same bytes
__global__ __launch_bounds__(256) void k_copy(const uint4 *src, uint4 *dst, long n) {
    const long st = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += st) dst[i] = src[i];
}

int main() {
    const long M = 4096, P = 4096;
    const long slot_bytes = 2 * (M + 2) * (P + 2) * 8;
    const long n = slot_bytes / 16;
    uint4 *arr[2];
    for (auto &p : arr) {
        CK(hipMalloc(&p, 3 * slot_bytes));
        CK(hipMemset(p, 1, 3 * slot_bytes));
    }
    uint4 *scratch;
    CK(hipMalloc(&scratch, 4 * slot_bytes));
    A a{{arr[0], arr[1]}, n};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 2.0 * 4 * slot_bytes;  // 2 arrays x (2 reads + 2 writes) x slot
    auto timeit = [&](const char *name, auto launch) {
        for (int w = 0; w < 5; ++w) launch();
        (void)hipEventRecord(e0);
        const int R = 20;
        for (int r = 0; r < R; ++r) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= R;
        std::printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; ++rep) {
        for (unsigned g : {2048u, 8192u, 32768u})
            timeit(g == 2048 ? "stride 2048 wg" : g == 8192 ? "stride 8192 wg" : "stride 32768 wg",
                   [&]() { k_stride<<<dim3(g, 2), 256>>>(a); });
        timeit("batch V=1", [&]() { k_batch<1><<<dim3((n + 255) / 256, 2), 256>>>(a); });
        timeit("batch V=2", [&]() { k_batch<2><<<dim3((n + 511) / 512, 2), 256>>>(a); });
        timeit("batch V=4", [&]() { k_batch<4><<<dim3((n + 1023) / 1024, 2), 256>>>(a); });
        timeit("batch V=4 nt", [&]() { k_batch_nt<4><<<dim3((n + 1023) / 1024, 2), 256>>>(a); });
        timeit("batch V=1 nt", [&]() { k_batch_nt<1><<<dim3((n + 255) / 256, 2), 256>>>(a); });
        timeit("memcpy x4 (3<-2, 2<-1)", [&]() {
            for (int k = 0; k < 2; ++k) {
                (void)hipMemcpyAsync(arr[k] + 2 * n, arr[k] + n, slot_bytes, hipMemcpyDeviceToDevice, 0);
                (void)hipMemcpyAsync(arr[k] + n, arr[k], slot_bytes, hipMemcpyDeviceToDevice, 0);
            }
        });
        timeit("plain copy 2x2 slots", [&]() {
            k_copy<<<8192, 256>>>(arr[0], scratch, 2 * n);
            k_copy<<<8192, 256>>>(arr[1], scratch + 2 * n, 2 * n);
        });
    }
    return 0;
}
