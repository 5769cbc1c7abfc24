// Diagnostic: does the tendency's strip walk lose bandwidth to its address spread?  Same
// 4-read / 2-write streaming mix as strip_stream.hip, 256-wide strips walking contiguous row
// ranges (two chip-fulls of workgroups, as the tendency at 4096^2), over three layouts:
//   row-major   the reference layout (rows of M+2 doubles, x contiguous)
//   strip-major each 256-column strip stored contiguously ([strip][row][256])
//   interleave  row-major, workgroup y takes rows y, y+ny, ... (all workgroups sweep together)
// Reports TB/s of the 6 algorithmic streams.
#include <hip/hip_runtime.h>
#include <cstdio>

enum { ROWMAJOR = 0, STRIPMAJOR = 1, INTERLEAVE = 2 };

template <int MODE>
__global__ __launch_bounds__(256) void walk(const double *__restrict__ a, const double *__restrict__ b,
                                            const double *__restrict__ c, const double *__restrict__ d,
                                            double *__restrict__ o1, double *__restrict__ o2, int M, int P, int ny) {
    const int j0 = (int)((long)blockIdx.y * P / ny), j1 = (int)((long)(blockIdx.y + 1) * P / ny);
    const size_t ld = M + 2, plane = ld * (P + 2);
    const size_t L = (size_t)blockIdx.z * plane;
    for (int jj = j0; jj < j1; ++jj) {
        const int j = MODE == INTERLEAVE ? (int)blockIdx.y + (jj - j0) * ny : jj;
        if (j >= P) break;
        size_t o;
        if (MODE == STRIPMAJOR) o = L + ((size_t)blockIdx.x * (P + 2) + (j + 1)) * 256 + threadIdx.x;
        else o = L + (size_t)(j + 1) * ld + blockIdx.x * 256 + threadIdx.x + 1;
        const double x = a[o], y = b[o], z = c[o], w = d[o];
        o1[o] = x + y;
        o2[o] = z * w;
    }
}

template <int MODE>
void run(const char *name, double **p, int M, int P, hipEvent_t e0, hipEvent_t e1) {
    for (int blocks : {1280, 2560, 5120}) {
        const int nx = M / 256, ny = blocks / (2 * nx) > 0 ? blocks / (2 * nx) : 1;
        float best = 1e9, sum = 0;
        int n = 0;
        for (int rep = 0; rep < 12; ++rep) {
            (void)hipEventRecord(e0);
            walk<MODE><<<dim3(nx, ny, 2), 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P, ny);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 1) { best = ms < best ? ms : best; sum += ms; ++n; }
        }
        const double bytes = 6.0 * M * P * 2 * 8;
        printf("%-11s rows/wg %4d wgs %5d: best %.3f ms %.2f TB/s  mean %.3f ms %.2f TB/s\n", name, P / ny,
               nx * ny * 2, best, bytes / (best * 1e-3) / 1e12, sum / n, bytes / (sum / n * 1e-3) / 1e12);
    }
}

int main() {
    const int M = 4096, P = 4096;
    const size_t F = (size_t)(M + 2) * (P + 2) * 2;
    double *p[6];
    for (auto &q : p) {
        if (hipMalloc(&q, F * 8) != hipSuccess) return 1;
        (void)hipMemset(q, 0, F * 8);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int round = 0; round < 2; ++round) {
        run<ROWMAJOR>("row-major", p, M, P, e0, e1);
        run<STRIPMAJOR>("strip-major", p, M, P, e0, e1);
        run<INTERLEAVE>("interleave", p, M, P, e0, e1);
    }
    for (auto &q : p) (void)hipFree(q);
    return 0;
}
