// Streaming ceiling for the tendency's access mix (read 4 fields, write 2), 8 B vs 16 B per
// lane, 16.8 M doubles per field.  hipcc --offload-arch=gfx950 -O3 stream_width.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W>  // doubles per lane per access
__global__ __launch_bounds__(256) void mix(const double *__restrict__ a, const double *__restrict__ b,
                                           const double *__restrict__ c, const double *__restrict__ d,
                                           double *__restrict__ o1, double *__restrict__ o2, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * W;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * W; i < n; i += stride) {
        if constexpr (W == 1) {
            const double x = a[i], y = b[i], z = c[i], w = d[i];
            o1[i] = x + y * z;
            o2[i] = w - x;
        } else {
            const double2 x = *(const double2 *)(a + i), y = *(const double2 *)(b + i);
            const double2 z = *(const double2 *)(c + i), w = *(const double2 *)(d + i);
            *(double2 *)(o1 + i) = make_double2(x.x + y.x * z.x, x.y + y.y * z.y);
            *(double2 *)(o2 + i) = make_double2(w.x - x.x, w.y - x.y);
        }
    }
}

int main() {
    const size_t n = 4096ull * 4096 * 2;  // both layers
    double *p[6];
    for (auto &q : p) {
        hipMalloc(&q, n * 8);
        hipMemset(q, 0, n * 8);
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int grid : {2048, 8192, 32768}) {
        for (int w : {1, 2}) {
            float best = 1e9;
            for (int rep = 0; rep < 10; ++rep) {
                hipEventRecord(e0);
                if (w == 1) mix<1><<<grid, 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], n);
                else mix<2><<<grid, 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], n);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 1 && ms < best) best = ms;
            }
            printf("grid %6d  %2d B/lane: %.3f ms  %.2f TB/s\n", grid, 8 * w, best, 6.0 * n * 8 / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
