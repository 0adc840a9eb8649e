// Micro-probe of VALU issue on gfx950 (diagnostic, not product code): cycles
// per v_fma_f32 for one or two waves per SIMD, full or half exec mask, and
// independent vs dependent chains.  Each workgroup is one wave; the grid puts
// `wps` waves on each SIMD (256 CUs x 4 SIMDs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <bool DEP>
__global__ __launch_bounds__(64) void k_fma(float *out, int iters, int active, long long *cyc) {
    if ((int)threadIdx.x >= active) return;
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 0.999f, c = 0.001f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if (DEP) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                a0 = fmaf(a0, m, c);
            }
        } else {
            a0 = fmaf(a0, m, c); a1 = fmaf(a1, m, c); a2 = fmaf(a2, m, c); a3 = fmaf(a3, m, c);
            a4 = fmaf(a4, m, c); a5 = fmaf(a5, m, c); a6 = fmaf(a6, m, c); a7 = fmaf(a7, m, c);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int iters = 20000;
    const int nwg_max = 256 * 4 * 4;
    float *out;
    long long *cyc;
    hipMalloc(&out, nwg_max * 64 * sizeof(float));
    hipMalloc(&cyc, nwg_max * sizeof(long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int dep = 0; dep < 2; dep++)
        for (int wps : {1, 2, 4})
            for (int active : {64, 32, 16}) {
                int nwg = 256 * 4 * wps;
                for (int rep = 0; rep < 2; rep++) {
                    hipEventRecord(e0);
                    if (dep)
                        k_fma<true><<<nwg, 64>>>(out, iters, active, cyc);
                    else
                        k_fma<false><<<nwg, 64>>>(out, iters, active, cyc);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                }
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                std::vector<long long> c(nwg);
                hipMemcpy(c.data(), cyc, nwg * sizeof(long long), hipMemcpyDeviceToHost);
                double avg = 0;
                for (auto v : c) avg += v;
                avg /= nwg;
                double instrs = 8.0 * iters;
                // chip-wide: wave-instrs per SIMD = wps * instrs over ms
                double cyc_per_instr_wall = ms * 1e-3 * 2.4e9 / (wps * instrs);
                printf("{\"dep\": %d, \"waves_per_simd\": %d, \"active_lanes\": %d, \"ms\": %.4f, "
                       "\"memtime_per_instr_per_wave\": %.3f, \"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
                       dep, wps, active, ms, avg / instrs, cyc_per_instr_wall);
            }
    return 0;
}
