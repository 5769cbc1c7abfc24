// Cost of a grid-wide barrier (cooperative launch, cooperative_groups grid.sync()) against a
// kernel boundary on the same stream, at the geometry of the 4096^2 spectral passes (256
// workgroups of 512 threads, one per CU).  Question it answers: can folding spec_carry into
// pass A's tail behind a grid barrier beat the separate launch?
//   hipcc -O3 --offload-arch=gfx950 grid_sync.hip -o grid_sync && ./grid_sync
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>

namespace cg = cooperative_groups;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                          \
        }                                                                      \
    } while (0)

// nsync grid barriers, a little work between them
__global__ __launch_bounds__(512) void k_sync(double *buf, int nsync) {
    cg::grid_group g = cg::this_grid();
    double v = buf[blockIdx.x * 512 + threadIdx.x];
    for (int s = 0; s < nsync; ++s) {
        v = v * 1.0000001 + 1e-9;
        g.sync();
    }
    buf[blockIdx.x * 512 + threadIdx.x] = v;
}

// the same work, one kernel per step (a kernel boundary instead of the barrier)
__global__ __launch_bounds__(512) void k_step(double *buf) {
    double v = buf[blockIdx.x * 512 + threadIdx.x];
    v = v * 1.0000001 + 1e-9;
    buf[blockIdx.x * 512 + threadIdx.x] = v;
}

int main() {
    int dev = 0, cus = 0, per = 0, coop = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_sync, 512, 100 * 1024));
    std::printf("CUs %d, cooperative launch %d, blocks/CU at 100 KB LDS %d\n", cus, coop, per);
    const int G = cus;  // one workgroup per CU, like the 4096^2 passes
    double *buf;
    CK(hipMalloc(&buf, sizeof(double) * G * 512));
    CK(hipMemset(buf, 0, sizeof(double) * G * 512));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        for (int nsync : {1, 100}) {
            int ns = nsync;
            void *args[] = {&buf, &ns};
            CK(hipLaunchCooperativeKernel((const void *)k_sync, dim3(G), dim3(512), args, 100 * 1024, 0));
            CK(hipEventRecord(e0));
            for (int r = 0; r < 10; ++r)
                CK(hipLaunchCooperativeKernel((const void *)k_sync, dim3(G), dim3(512), args, 100 * 1024, 0));
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("cooperative kernel with %3d grid barriers: %8.2f us per kernel\n", nsync, ms * 1e3 / 10);
        }
        CK(hipEventRecord(e0));
        for (int r = 0; r < 100; ++r) k_step<<<G, 512, 100 * 1024>>>(buf);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("100 back-to-back kernels: %8.2f us per kernel (boundary + launch)\n", ms * 1e3 / 100);
    }
    return 0;
}
