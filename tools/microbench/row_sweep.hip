// Diagnostic: a tendency-like access pattern WITHOUT LDS rings -- one workgroup per output
// row (all workgroups sweep the field together), each reading 5 rows of a (psi), 3 of b
// (zeta), 1 of c, d (F history) with x-neighbours, writing 2 rows: vertical reuse is left
// to the caches.  XCD = 1 maps consecutive rows to the same XCD (workgroup w runs on XCD
// w % 8), so the 5-row window is shared in that XCD's L2.  Reports algorithmic TB/s
// (6 words per point) -- compare with the ring-based strips (4.3-4.7 TB/s).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int TPB, int XCD>
__global__ __launch_bounds__(TPB) void rows(const double *__restrict__ a, const double *__restrict__ b,
                                            const double *__restrict__ c, const double *__restrict__ d,
                                            double *__restrict__ o1, double *__restrict__ o2, int M, int P) {
    const int w = blockIdx.x;
    int j;
    if (XCD) {
        const int per = P / 8;  // rows per XCD band
        j = (w % 8) * per + w / 8;
    } else {
        j = w;
    }
    const size_t ld = M + 2, L = (size_t)blockIdx.y * ld * (P + 2);
    auto at = [&](const double *p, int jj, int i) {  // periodic rows via clamp-free wrap
        jj = jj < 0 ? jj + P : (jj >= P ? jj - P : jj);
        return p[L + (size_t)(jj + 1) * ld + i + 1];
    };
    for (int i = threadIdx.x; i < M; i += TPB) {
        const int im = i > 0 ? i - 1 : M - 1, ip = i + 1 < M ? i + 1 : 0;
        double s = 0;
#pragma unroll
        for (int dj = -2; dj <= 2; ++dj) s += at(a, j + dj, i);
        s += at(a, j, im) + at(a, j, ip);
        double z = at(b, j - 1, i) + at(b, j, i) + at(b, j + 1, i) + at(b, j, im) + at(b, j, ip);
        const size_t o = L + (size_t)(j + 1) * ld + i + 1;
        o1[o] = s * z + c[o];
        o2[o] = s - z * d[o];
    }
}

template <int TPB, int XCD>
void run(double **p, int M, int P, hipEvent_t e0, hipEvent_t e1) {
    float best = 1e9;
    for (int rep = 0; rep < 10; ++rep) {
        (void)hipEventRecord(e0);
        rows<TPB, XCD><<<dim3(P, 2), TPB>>>(p[0], p[1], p[2], p[3], p[4], p[5], M, P);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 1 && ms < best) best = ms;
    }
    printf("TPB %4d XCD %d: %.3f ms  %.2f TB/s (algorithmic 6 words/pt)\n", TPB, XCD, best,
           6.0 * M * P * 2 * 8 / (best * 1e-3) / 1e12);
}

int main() {
    const int M = 4096, P = 4096;
    const size_t F = (size_t)(M + 2) * (P + 2) * 2;
    double *p[6];
    for (auto &q : p) {
        (void)hipMalloc(&q, F * 8);
        (void)hipMemset(q, 0, F * 8);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    run<256, 0>(p, M, P, e0, e1);
    run<256, 1>(p, M, P, e0, e1);
    run<512, 0>(p, M, P, e0, e1);
    run<512, 1>(p, M, P, e0, e1);
    run<1024, 0>(p, M, P, e0, e1);
    run<1024, 1>(p, M, P, e0, e1);
    return 0;
}
