// Diagnostic: the tendency's HBM access pattern without its LDS / arithmetic.  Strips of W
// columns (256 threads, W/256 columns each) x rows split over ny workgroups, 4 streams read and
// 2 written per point, rows of M+2 doubles at interior offset 1.  Reports TB/s.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W, bool INTERLEAVE>
__global__ __launch_bounds__(256) void strips(const double *__restrict__ a, const double *__restrict__ b,
                                              const double *__restrict__ c, const double *__restrict__ d,
                                              double *__restrict__ o1, double *__restrict__ o2, int M, int P, int ny) {
    const int j0 = (int)((long)blockIdx.y * P / ny), j1 = (int)((long)(blockIdx.y + 1) * P / ny);
    const size_t ld = M + 2, L = (size_t)blockIdx.z * ld * (P + 2);
    for (int jj = j0; jj < j1; ++jj) {
        // INTERLEAVE: workgroup y takes rows y, y + ny, ... (all workgroups sweep the field
        // together); else a contiguous range
        const int j = INTERLEAVE ? (int)blockIdx.y + (jj - j0) * ny : jj;
        if (j >= P) break;
#pragma unroll
        for (int q = 0; q < W / 256; ++q) {
            const int i = blockIdx.x * W + q * 256 + threadIdx.x;
            const size_t o = L + (size_t)(j + 1) * ld + i + 1;
            const double x = a[o], y = b[o], z = c[o], w = d[o];
            o1[o] = x + y;
            o2[o] = z * w;
        }
    }
}

template <int W, bool IL>
void run(double **p, int M, int P, hipEvent_t e0, hipEvent_t e1) {
    for (int blocks : {1280, 2560, 8192, 16384, 32768}) {
        const int nx = M / W, ny = blocks / (2 * nx) > 0 ? blocks / (2 * nx) : 1;
        float best = 1e9;
        for (int rep = 0; rep < 8; ++rep) {
            (void)hipEventRecord(e0);
            strips<W, IL><<<dim3(nx, ny, 2), 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P, ny);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 1 && ms < best) best = ms;
        }
        printf("W %4d IL %d blocks %5d: %.3f ms  %.2f TB/s\n", W, (int)IL, nx * ny * 2, best, 6.0 * M * P * 2 * 8 / (best * 1e-3) / 1e12);
    }
}

int main() {
    const int M = 4096, P = 4096;
    const size_t F = (size_t)(M + 2) * (P + 2) * 2;
    double *p[6];
    for (auto &q : p) { (void)hipMalloc(&q, F * 8); (void)hipMemset(q, 0, F * 8); }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    run<256, false>(p, M, P, e0, e1);
    run<512, false>(p, M, P, e0, e1);
    return 0;
}
