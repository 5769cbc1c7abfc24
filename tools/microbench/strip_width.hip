// Diagnostic (r04): the tendency's strip walk (4 streams read, 2 written per point, row ranges
// per workgroup, XCD order, the reference layout: interior at element 1 of rows of M + 2
// doubles) with wider accesses.  The ring streams (psi, zeta) are read once per row into LDS,
// so their per-lane width is free to choose; F(t-1), F(t-2) and the two outputs are pointwise.
//   ref8   : every access 8 B per lane (today's tendency: lane t <-> column x0 + t)
//   ring16 : psi and zeta rows read 16 B per lane (threads 0-127 psi, 128-255 zeta) and written
//            to an LDS row buffer (one barrier per row), F loads and stores 8 B per lane
//   dma16  : psi and zeta rows by LDS-DMA (global_load_lds_dwordx4), F and stores 8 B
//   all16  : two columns per lane, every access 16 B (256 threads, 512-column strips)
//   alig8  : ref8 over a 128-B aligned pitch (the bound for this walk; not the layout)
// hipcc --offload-arch=gfx950 -O3 strip_width.hip -o strip_width
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));

__device__ __forceinline__ int xcd_id() {
    const int W = gridDim.x * gridDim.y * gridDim.z;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int full = W - W % 8;
    return b < full ? (b % 8) * (full / 8) + b / 8 : b;
}

template <int MODE>  // 0 ref8, 1 ring16, 2 dma16, 3 all16, 4 alig8
__global__ __launch_bounds__(256) void walk(const double *__restrict__ a, const double *__restrict__ b,
                                            const double *__restrict__ c, const double *__restrict__ d,
                                            double *__restrict__ o1, double *__restrict__ o2, int M, int P,
                                            int ny, long ld, int off) {
    const int l = xcd_id();
    const int bx = l % gridDim.x, r = l / gridDim.x, by = r % gridDim.y, bz = r / gridDim.y;
    const int j0 = (int)((long)by * P / ny), j1 = (int)((long)(by + 1) * P / ny);
    const size_t L = (size_t)bz * ld * (P + 2);
    constexpr int W = MODE == 3 ? 512 : 256;
    const int x0 = bx * W, t = threadIdx.x;
    __shared__ __attribute__((aligned(16))) double ring[2][2][W + 8];
    double acc = 0;
    for (int j = j0; j < j1; ++j) {
        const size_t B = L + (size_t)(j + 1) * ld + off + x0;
        if constexpr (MODE == 0 || MODE == 4) {
            const double x = a[B + t], y = b[B + t], z = c[B + t], w = d[B + t];
            o1[B + t] = x + y + acc;
            o2[B + t] = z * w;
        } else if constexpr (MODE == 1 || MODE == 2) {
            double *rw = &ring[j & 1][t >> 7][0];
            const double *src = (t >> 7) ? b : a;
            const int q = t & 127;
            if constexpr (MODE == 1) {
                const d2u v = *(const d2u *)(src + B + 2 * q);
                *(double2 *)(rw + 2 * q) = make_double2(v.x, v.y);
            } else {
                __builtin_amdgcn_global_load_lds((const void *)(src + B + 2 * q), (__attribute__((address_space(3))) void *)(rw + 2 * (q & ~63)), 16, 0, 0);
            }
            const double z = c[B + t], w = d[B + t];
            if constexpr (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const double x = ring[j & 1][0][t], y = ring[j & 1][1][t];
            o1[B + t] = x + y + acc;
            o2[B + t] = z * w;
        } else {  // all16
            const d2u x = *(const d2u *)(a + B + 2 * t), y = *(const d2u *)(b + B + 2 * t);
            const d2u z = *(const d2u *)(c + B + 2 * t), w = *(const d2u *)(d + B + 2 * t);
            *(d2u *)(o1 + B + 2 * t) = x + y + acc;
            *(d2u *)(o2 + B + 2 * t) = z * w;
        }
    }
    if (acc == 12345.0) o1[0] = acc;
}

template <int MODE>
void run(double **p, int M, int P, long ld, int off, hipEvent_t e0, hipEvent_t e1, const char *name) {
    constexpr int W = MODE == 3 ? 512 : 256;
    for (int rows : {17, 34}) {
        const int nx = M / W, ny = P / rows * (W / 256);
        float best = 1e9, sum = 0;
        int cnt = 0;
        for (int rep = 0; rep < 12; ++rep) {
            (void)hipEventRecord(e0);
            walk<MODE><<<dim3(nx, ny, 2), 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P, ny, ld, off);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 1) {
                if (ms < best) best = ms;
                sum += ms;
                ++cnt;
            }
        }
        const double bytes = 6.0 * M * P * 2 * 8;
        printf("%-7s rows/wg %3d wgs %5d: best %.3f ms %.2f TB/s  mean %.3f ms\n", name, P / ny * (W / 256), nx * ny * 2, best,
               bytes / (best * 1e-3) / 1e12, sum / cnt);
    }
}

int main() {
    const int M = 4096, P = 4096;
    const size_t F = (size_t)(M + 16) * (P + 2) * 2 + 1024;
    double *p[6];
    for (auto &q : p) {
        (void)hipMalloc(&q, F * 8);
        (void)hipMemset(q, 0, F * 8);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int pass = 0; pass < 2; ++pass) {
        run<0>(p, M, P, M + 2, 1, e0, e1, "ref8");
        run<1>(p, M, P, M + 2, 1, e0, e1, "ring16");
        run<2>(p, M, P, M + 2, 1, e0, e1, "dma16");
        run<3>(p, M, P, M + 2, 1, e0, e1, "all16");
        run<4>(p, M, P, M + 16, 0, e0, e1, "alig8");
    }
    return 0;
}
