// Diagnostic: the tendency's F32 HBM access pattern (4 streams read, 2 written per point,
// strips of 256 threads x VEC points, contiguous row ranges) with VEC = 1 (one float per
// thread, as the F32 tendency) or 2 (float2 per thread, 4-byte aligned as interior rows are).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int VEC>
__global__ __launch_bounds__(256) void strips(const float *__restrict__ a, const float *__restrict__ b,
                                              const float *__restrict__ c, const float *__restrict__ d,
                                              float *__restrict__ o1, float *__restrict__ o2, int M, int P, int ny) {
    const int j0 = (int)((long)blockIdx.y * P / ny), j1 = (int)((long)(blockIdx.y + 1) * P / ny);
    const size_t ld = M + 2, L = (size_t)blockIdx.z * ld * (P + 2);
    for (int j = j0; j < j1; ++j) {
        const int i = (blockIdx.x * 256 + threadIdx.x) * VEC;
        const size_t o = L + (size_t)(j + 1) * ld + i + 1;
        if constexpr (VEC == 1) {
            const float x = a[o], y = b[o], z = c[o], w = d[o];
            o1[o] = x + y;
            o2[o] = z * w;
        } else {
            typedef float f2 __attribute__((ext_vector_type(2), aligned(4)));
            const f2 x = *(const f2 *)(a + o), y = *(const f2 *)(b + o), z = *(const f2 *)(c + o),
                     w = *(const f2 *)(d + o);
            *(f2 *)(o1 + o) = x + y;
            *(f2 *)(o2 + o) = z * w;
        }
    }
}

template <int VEC>
void run(float **p, int M, int P, hipEvent_t e0, hipEvent_t e1) {
    for (int blocks : {1280, 2560, 4096, 8192, 16384}) {
        const int nx = M / (256 * VEC), ny = blocks / (2 * nx) > 0 ? blocks / (2 * nx) : 1;
        float best = 1e9;
        for (int rep = 0; rep < 8; ++rep) {
            (void)hipEventRecord(e0);
            strips<VEC><<<dim3(nx, ny, 2), 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P, ny);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 1 && ms < best) best = ms;
        }
        printf("F32 VEC %d blocks %5d: %.3f ms  %.2f TB/s\n", VEC, nx * ny * 2, best,
               6.0 * M * P * 2 * 4 / (best * 1e-3) / 1e12);
    }
}

int main() {
    for (int M : {4096, 8192}) {
        const int P = M;
        const size_t F = (size_t)(M + 2) * (P + 2) * 2;
        float *p[6];
        for (auto &q : p) {
            (void)hipMalloc(&q, F * 4);
            (void)hipMemset(q, 0, F * 4);
        }
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        printf("M = %d\n", M);
        run<1>(p, M, P, e0, e1);
        run<2>(p, M, P, e0, e1);
        for (auto &q : p) (void)hipFree(q);
    }
    return 0;
}
