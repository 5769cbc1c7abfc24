"""Add wall_clock64 phase stamps to spec_passA_half (the wide-row pass A) in a COPY of csrc
(experiment builds only): python tools/stamps/add_stamps_half.py DIR.  Read back with
tools/stamps/stamps_passA_half.py.  Per workgroup 256 slots: 0 entry, 1 rows start, then five
per row (row start, projection done = prefetched row arrived, hook = stage 1 + T1 writes done,
transform done, split + recurrence + u stores issued), 255 exit after the stores drained."""
import sys

p = sys.argv[1] + '/qg_spectral.hip'
s = open(p).read()
rep = [
    ('''namespace qg {

constexpr int CARRY_WAVES = 8;''', '''namespace qg {
__device__ unsigned long long g_stamp[1024 * 256];
#define STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < 1024) { unsigned long long _t = wall_clock64(); __builtin_nontemporal_store(_t, &g_stamp[blockIdx.x * 256 + (slot)]); } } while (0)

constexpr int CARRY_WAVES = 8;'''),
]
a0, b0 = rep[0]
assert s.count(a0) == 1
s = s.replace(a0, b0)
i0 = s.index('__global__ __launch_bounds__(HT, 2) void spec_passA_half(SpecArgs a) {')
i1 = s.index('// SYS 0: psi~1 (pinned) -> half_tmp')
seg = s[i0:i1]
body = [
    ('''    half_lds_init(a, tw512);
    __syncthreads();''', '''    STAMP(0);
    half_lds_init(a, tw512);
    __syncthreads();'''),
    ('''        if constexpr (!RQ_HOIST) asm volatile("" ::: "memory");  // keep coefficient loads in the loop''',
     '''        const int rs_ = 2 + 5 * (e - j);
        STAMP(rs_);
        if constexpr (!RQ_HOIST) asm volatile("" ::: "memory");  // keep coefficient loads in the loop'''),
    ('''        const int tt = opaque_tid();
        lx::fft<false, false, true>(in, b0, b1, tw512, tt, [&]() {
            if (jn >= s0) load_row(jn, c1, c2);
        });''', '''        asm volatile("" ::"v"(in[0].x), "v"(in[7].y));
        STAMP(rs_ + 1);
        const int tt = opaque_tid();
        lx::fft<false, false, true>(in, b0, b1, tw512, tt, [&]() {
            STAMP(rs_ + 2);
            if (jn >= s0) load_row(jn, c1, c2);
        }, s2f);
        asm volatile("" ::"v"(in[0].x), "v"(in[7].y));
        STAMP(rs_ + 3);'''),
    ('''                bw[q] = cfma(om[q].x, u[q], bw[q]);
                om[q].x *= r;
            }
        }
    };''', '''                bw[q] = cfma(om[q].x, u[q], bw[q]);
                om[q].x *= r;
            }
        }
        STAMP(rs_ + 4);
    };'''),
    ('''    load_row(e, pf1, pf2);
    for (int j = e; j >= s0; --j) row_step(j, pf1, pf2, j - 1);''', '''    load_row(e, pf1, pf2);
    STAMP(1);
    for (int j = e; j >= s0; --j) row_step(j, pf1, pf2, j - 1);'''),
    ('''    if (t == 0 && s == 0) a.dcpart[c] = dc;
}''', '''    if (t == 0 && s == 0) a.dcpart[c] = dc;
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(255);
}'''),
]
for a, b in body:
    assert seg.count(a) == 1, a[:70]
    seg = seg.replace(a, b)
s = s[:i0] + seg + s[i1:]
s += '''
extern "C" int qg_debug_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(qg::g_stamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
'''
open(p, 'w').write(s)
