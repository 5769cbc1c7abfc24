// Diagnostic: does the tendency's strip walk lose HBM rate to misaligned rows?  The reference
// layout puts interior column 0 at element 1 of a row of M + 2 doubles, so a wave's 64-lane
// 8-byte access spans 5 cache lines (128 B) instead of 4 on most rows, and neighbouring strips
// share (and partially write) the line at their common edge.  Same 4-read / 2-write mix and
// strip walk as strip_stream.hip (256 threads, one double per lane, row ranges per
// workgroup).  Address patterns:
//   ref   : ld = M + 2, interior offset 1 (the reference layout, lane t -> column x0 + t)
//   alig  : ld = M + 16, offset 0 (every row 128-B aligned: the best case, not the layout)
//   rot   : reference layout, lane t -> column x0 + (t + d_j) mod 256 (d_j: the row's leading
//           partial line), so waves 0-2 touch 4 lines and wave 3 five (17 vs 20)
//   cut128/cut64: reference layout, the strip's row segment starts at the first 128-B (64-B)
//           boundary at or after column x0 (cut points drift with the row; every line written
//           by one workgroup)
//   rotoff1/2: rot with one / two of the read streams 64 B off the line phase of the others
//   rotwoff: rot with one of the two written streams 64 B off the line phase
//   rot64 : rot at 64-B granularity (d_j: the row's leading partial 64-B segment)
//   hyb64 : the tendency's form of cut64: two streams (psi, zeta rings) read as an aligned
//           window of 256 + 16 elements from the 64-B boundary at or before column x0 - 2,
//           the other two reads and both writes at the cut64 columns
// XCD: the tendency's xcd_logical_id workgroup order (contiguous logical ranges per XCD).
// hipcc --offload-arch=gfx950 -O3 strip_align.hip -o strip_align
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int xcd_id() {
    const int W = gridDim.x * gridDim.y * gridDim.z;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int full = W - W % 8;
    return b < full ? (b % 8) * (full / 8) + b / 8 : b;
}

template <int MODE, bool XCD>  // 0 ref, 1 alig, 2 rot, 3 cut128, 4 cut64, 5 hyb64, 6/7 rot with 1/2 reads 64 B off phase,
          // 8 rot with one write 64 B off phase, 9 rot at 64-B granularity
__global__ __launch_bounds__(256) void walk(const double *__restrict__ a, const double *__restrict__ b,
                                            const double *__restrict__ c, const double *__restrict__ d,
                                            double *__restrict__ o1, double *__restrict__ o2, int M, int P,
                                            int ny, long ld, int off) {
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (XCD) {
        const int l = xcd_id();
        bx = l % gridDim.x;
        const int r = l / gridDim.x;
        by = r % gridDim.y;
        bz = r / gridDim.y;
    }
    const int j0 = (int)((long)by * P / ny), j1 = (int)((long)(by + 1) * P / ny);
    const size_t L = (size_t)bz * ld * (P + 2);
    const int x0 = bx * 256, t = threadIdx.x;
    double acc = 0;
    for (int j = j0; j < j1; ++j) {
        const size_t B = L + (size_t)(j + 1) * ld + off + x0;
        size_t o = B + t;
        if (MODE == 2 || (MODE >= 6 && MODE <= 8)) o = B + ((t + (int)((16 - (B & 15)) & 15)) & 255);
        if (MODE == 9) o = B + ((t + (int)((8 - (B & 7)) & 7)) & 255);
        if (MODE == 3) o = ((B + 15) & ~(size_t)15) + t;
        if (MODE == 4 || MODE == 5) o = ((B + 7) & ~(size_t)7) + t;
        if (MODE == 5) {
            const size_t w0 = (B - 2) & ~(size_t)7;
            const double x = a[w0 + t], y = b[w0 + t];
            double x2 = 0, y2 = 0;
            if (t < 16) {
                x2 = a[w0 + 256 + t];
                y2 = b[w0 + 256 + t];
            }
            const double z = c[o], w = d[o];
            o1[o] = x + y + acc;
            o2[o] = z * w;
            acc = x2 + y2;
        } else {
            // MODE 6 / 7: the third (and fourth) stream sits 64 B off the others' line phase (the
            // state's slots differ by 64 B mod 128), read with the same lane mapping
            const double x = a[o], y = b[o], z = c[o + (MODE >= 6 ? 8 : 0)], w = d[o + (MODE == 7 ? 8 : 0)];
            o1[o] = x + y;
            o2[o + (MODE == 8 ? 8 : 0)] = z * w;
        }
    }
    if (acc == 12345.0) o1[0] = acc;
}

template <int MODE, bool XCD>
void run(double **p, int M, int P, long ld, int off, hipEvent_t e0, hipEvent_t e1, const char *name) {
    for (int rows : {17, 34, 68}) {
        const int nx = M / 256, ny = P / rows;
        float best = 1e9, sum = 0;
        int cnt = 0;
        for (int rep = 0; rep < 12; ++rep) {
            (void)hipEventRecord(e0);
            walk<MODE, XCD><<<dim3(nx, ny, 2), 256>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P, ny, ld, off);
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
        printf("%-6s xcd %d rows/wg %3d wgs %5d: best %.3f ms %.2f TB/s  mean %.3f ms %.2f TB/s\n", name, (int)XCD, rows,
               nx * ny * 2, best, bytes / (best * 1e-3) / 1e12, sum / cnt, bytes / (sum / cnt * 1e-3) / 1e12);
    }
}

template <bool X>
void all(double **p, int M, int P, hipEvent_t e0, hipEvent_t e1) {
    run<0, X>(p, M, P, M + 2, 1, e0, e1, "ref");
    run<1, X>(p, M, P, M + 16, 0, e0, e1, "alig");
    run<2, X>(p, M, P, M + 2, 1, e0, e1, "rot");
    run<3, X>(p, M, P, M + 2, 1, e0, e1, "cut128");
    run<4, X>(p, M, P, M + 2, 1, e0, e1, "cut64");
    run<5, X>(p, M, P, M + 2, 1, e0, e1, "hyb64");
    run<6, X>(p, M, P, M + 2, 1, e0, e1, "rotoff1");
    run<7, X>(p, M, P, M + 2, 1, e0, e1, "rotoff2");
    run<8, X>(p, M, P, M + 2, 1, e0, e1, "rotwoff");
    run<9, X>(p, M, P, M + 2, 1, e0, e1, "rot64");
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
        all<true>(p, M, P, e0, e1);
    }
    return 0;
}
