/* run_model_no_output (src/run_model_no_output.jl:3-16) driven from plain C through the
 * C-ABI of include/qg_mi355.h: no Python, no torch -- device memory from the HIP runtime,
 * the default stream, the benchmark parameters of src/benchmarking/julia_bench_parts.jl:6-18.
 *
 *   run_no_output M P steps [solver(0 spectral | 1 pcg)] [out.bin]
 *
 * Prints one JSON line (diagnostics of the final state); with out.bin, also writes the final
 * zeta and psi (slot 1, both layers, ghost ring included: 2 x (M+2)(P+2) doubles each, Julia
 * column-major order) for a bitwise comparison with another driver.                      */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "qg_mi355.h"

#define CHECK(x)                                                                        \
    do {                                                                                \
        int s_ = (x);                                                                   \
        if (s_ != 0) {                                                                  \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, s_, qg_strerror(s_));           \
            return 1;                                                                   \
        }                                                                               \
    } while (0)
#define HCHECK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s M P steps [solver] [out.bin]\n", argv[0]);
        return 2;
    }
    const long M = atol(argv[1]), P = atol(argv[2]), steps = atol(argv[3]);
    const int solver = argc > 4 ? atoi(argv[4]) : QG_SOLVER_SPECTRAL;
    const char *out = argc > 5 ? argv[5] : NULL;
    if (qg_abi_version() != QG_ABI_VERSION) {
        fprintf(stderr, "ABI mismatch\n");
        return 1;
    }
    qg_params p;
    qg_default_params(&p); /* P_fwd = P_matrix(H_1, H_1) as model.jl:173 */
    const double KM = 1000.0, Lx = 4000.0 * KM;
    p.H_1 = 1.0 * KM;
    p.H_2 = 2.0 * KM;
    p.beta = 2e-11;
    p.Lx = Lx;
    p.Ly = Lx * (double)P / (double)M;
    p.dt = 30.0 * 60.0;
    p.T = 86400.0;
    p.U = 0.1;
    p.M = M;
    p.P = P;
    p.dx = Lx / (double)M;
    p.visc = 100.0;
    p.r = 1e-7;
    p.R_d = 40.0 * KM;
    p.initial_kick = 1e-6;
    p.solver = solver;

    qg_ctx *ctx = NULL;
    CHECK(qg_create(&p, 0, NULL, &ctx));
    const size_t field = (size_t)(M + 2) * (size_t)(P + 2), bytes = sizeof(double) * field * 6;
    double *zeta, *psi, *f_store;
    HCHECK(hipMalloc((void **)&zeta, bytes));
    HCHECK(hipMalloc((void **)&psi, bytes));
    HCHECK(hipMalloc((void **)&f_store, bytes));
    CHECK(qg_bind_state(ctx, zeta, psi, f_store));
    CHECK(qg_initialise(ctx, 20241008ULL, 20241009ULL));
    CHECK(qg_run(ctx, 1, steps));
    CHECK(qg_canonicalize(ctx)); /* newest state back in slot 1 */
    qg_diag d;
    CHECK(qg_diagnostics(ctx, &d));
    int it_p = 0, it_h = 0;
    double rr_p = 0, rr_h = 0;
    CHECK(qg_solver_stats(ctx, &it_p, &it_h, &rr_p, &rr_h));
    printf("{\"M\": %ld, \"P\": %ld, \"steps\": %ld, \"solver\": %d, \"psi_max\": [%.17g, %.17g], "
           "\"psi_min\": [%.17g, %.17g], \"zeta_sum\": [%.17g, %.17g], \"energy\": [%.17g, %.17g], "
           "\"pcg_iters\": [%d, %d]}\n",
           M, P, steps, solver, d.psi_max[0], d.psi_max[1], d.psi_min[0], d.psi_min[1], d.zeta_sum[0], d.zeta_sum[1],
           d.energy[0], d.energy[1], it_p, it_h);
    if (out) {
        double *h = (double *)malloc(sizeof(double) * field * 4);
        if (!h) return 1;
        HCHECK(hipMemcpy(h, zeta, sizeof(double) * field * 2, hipMemcpyDeviceToHost)); /* zeta[:,:,:,1] */
        HCHECK(hipMemcpy(h + 2 * field, psi, sizeof(double) * field * 2, hipMemcpyDeviceToHost));
        FILE *f = fopen(out, "wb");
        if (!f || fwrite(h, sizeof(double), field * 4, f) != field * 4) return 1;
        fclose(f);
        free(h);
    }
    CHECK(qg_destroy(ctx));
    HCHECK(hipFree(zeta));
    HCHECK(hipFree(psi));
    HCHECK(hipFree(f_store));
    return 0;
}
