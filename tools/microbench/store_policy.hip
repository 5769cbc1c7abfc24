// Store cache policy of a streaming writer and the kernel boundary behind it (r04).  A kernel
// that leaves B dirty bytes in the XCDs' L2s pays for their write-back at its end; stores that
// write through (sc1) or bypass (nt) leave none.  Each variant: a copy kernel (read 2 fields,
// write 2 fields, 16 B per lane, or 8 B per lane at the reference row offset like the
// tendency), then a dependent reader of what it wrote; HIP events around the writer alone and
// the pair.
//   hipcc -O3 --offload-arch=gfx950 store_policy.hip -o store_policy && ./store_policy
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));

template <int AUX>
__device__ __forceinline__ void st16(double2 *base, long i, double2 v, __amdgpu_buffer_rsrc_t r) {
    if constexpr (AUX < 0) {
        base[i] = v;
    } else {
        i4v w = __builtin_bit_cast(i4v, v);
        __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(i * 16), 0, AUX);
    }
}
template <int AUX>
__device__ __forceinline__ void st8(double *base, long i, double v, __amdgpu_buffer_rsrc_t r) {
    if constexpr (AUX < 0) {
        base[i] = v;
    } else {
        i2v w = __builtin_bit_cast(i2v, v);
        __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)(i * 8), 0, AUX);
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void *p, long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

// 16 B per lane, grid-stride
template <int AUX>
__global__ __launch_bounds__(256) void copy16(const double2 *a, const double2 *b, double2 *c, double2 *d, long n) {
    const auto rc = rsrc(c, n * 16), rd = rsrc(d, n * 16);
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const double2 x = a[i], y = b[i];
        st16<AUX>(c, i, make_double2(x.x + y.x, x.y + y.y), rc);
        st16<AUX>(d, i, make_double2(x.x * y.x, x.y * y.y), rd);
    }
}

// 8 B per lane, rows of M + 2 doubles, interior from element 1 (the reference layout)
template <int AUX>
__global__ __launch_bounds__(256) void copy8row(const double *a, const double *b, double *c, double *d, int M, int P) {
    const long ld = M + 2, bytes = ld * (P + 2) * 8;
    const auto rc = rsrc(c, bytes), rd = rsrc(d, bytes);
    for (int j = blockIdx.y; j < P; j += gridDim.y) {
        const long o = (long)(j + 1) * ld + 1 + blockIdx.x * 256 + threadIdx.x;
        const double x = a[o], y = b[o];
        st8<AUX>(c, o, x + y, rc);
        st8<AUX>(d, o, x * y, rd);
    }
}

__global__ __launch_bounds__(256) void reader(const double *c, const double *d, long n, double *out) {
    double s = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += c[i] + d[i];
    if (s == 12345.678) out[0] = s;  // (never: keeps the loads)
}

int main() {
    const int M = 4096, P = 4096;
    const long n16 = (long)M * P / 2 * 2;  // 268 MB per field as double2
    const long nd = (long)(M + 2) * (P + 2) * 2;
    double *f[5];
    for (auto &p : f) {
        (void)hipMalloc(&p, nd * 8 + 4096);
        (void)hipMemset(p, 0, nd * 8 + 4096);
    }
    hipEvent_t e0, e1, e2;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventCreate(&e2);
    const double gb = 4.0 * n16 * 16 / 1e9;
    auto run = [&](const char *name, auto launch) {
        float bw = 1e9, bp = 1e9, br = 1e9;
        for (int rep = 0; rep < 12; ++rep) {
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            reader<<<2048, 256>>>(f[2], f[3], n16 * 2, f[4]);
            (void)hipEventRecord(e2);
            (void)hipEventSynchronize(e2);
            float w, p;
            (void)hipEventElapsedTime(&w, e0, e1);
            (void)hipEventElapsedTime(&p, e0, e2);
            if (rep > 2) {
                bw = w < bw ? w : bw;
                bp = p < bp ? p : bp;
                br = (p - w) < br ? (p - w) : br;
            }
        }
        std::printf("%-22s writer %.3f ms (%.2f TB/s)  reader %.3f ms  pair %.3f ms\n", name, bw, gb / bw / 1e3, br, bp);
    };
    const auto A = (const double2 *)f[0], B = (const double2 *)f[1];
    auto C = (double2 *)f[2], D = (double2 *)f[3];
    for (int g : {1024, 4096}) {
        std::printf("grid %d\n", g);
        run("16B plain", [&] { copy16<-1><<<g, 256>>>(A, B, C, D, n16); });
        run("16B buffer aux0", [&] { copy16<0><<<g, 256>>>(A, B, C, D, n16); });
        run("16B sc1", [&] { copy16<16><<<g, 256>>>(A, B, C, D, n16); });
        run("16B nt", [&] { copy16<2><<<g, 256>>>(A, B, C, D, n16); });
        run("16B sc0 sc1", [&] { copy16<17><<<g, 256>>>(A, B, C, D, n16); });
    }
    const dim3 gr(M / 256, 512);
    run("8B row plain", [&] { copy8row<-1><<<gr, 256>>>(f[0], f[1], f[2], f[3], M, P); });
    run("8B row sc1", [&] { copy8row<16><<<gr, 256>>>(f[0], f[1], f[2], f[3], M, P); });
    run("8B row nt", [&] { copy8row<2><<<gr, 256>>>(f[0], f[1], f[2], f[3], M, P); });
    return 0;
}
