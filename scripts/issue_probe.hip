// Micro-probe of VALU issue on gfx950 (diagnostic, not product code): cycles
// per instruction of one wave's stream for 1, 2 and 4 waves per SIMD.  Each
// workgroup is one 64-lane wave that reserves LDS so that exactly `wps`
// workgroups fit per SIMD (4 * wps per CU) and the grid is 1024 * wps
// workgroups: the waves cannot stack on a SIMD.  Per-wave cycles come from
// s_memtime (the shader clock) around the loop.
//   fma      8 independent v_fma_f32 chains
//   pk_fma   8 independent v_pk_fma_f32 chains (16 FMAs per 8 instructions)
//   dep      one dependent v_fma_f32 chain
//   dpp      v_add_f32 with a DPP quad_perm source, 8 independent chains
//   fmac_e32 8 independent v_fmac_f32_e32 chains (the 32-bit VOP2 encoding)
//   acc_read 8 independent v_accvgpr_read_b32 (AGPR -> VGPR moves)
//   fmac_lit v_fmac_f32 with a literal constant (VOP2 + 32-bit literal)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float float2_t __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(64) void k_probe(float *out, int iters, long long *cyc) {
    extern __shared__ float lds[];
    float a[8];
    float2_t p[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        a[k] = threadIdx.x + k;
        p[k] = float2_t{(float)threadIdx.x + k, (float)threadIdx.x - k};
    }
    const float m = 0.999f, c = 0.001f;
    const float2_t m2 = {0.999f, 0.998f}, c2 = {0.001f, 0.002f};
    long long t0 = __builtin_amdgcn_s_memtime();
    // 16 x 8 instructions per trip: the loop's own branch (a taken branch
    // refetches the instruction stream) costs a lone wave ~30 cycles and must
    // not be what is measured
    for (int i = 0; i < iters; i++)
#pragma unroll
    for (int rr = 0; rr < 16; rr++) {
        if constexpr (KIND == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(m), "v"(c));
        } else if constexpr (KIND == 1) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[k]) : "v"(m2), "v"(c2));
        } else if constexpr (KIND == 2) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(m), "v"(c));
        } else if constexpr (KIND == 3) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_add_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                             : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
        } else if constexpr (KIND == 4) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[k]) : "v"(m), "v"(c));
        } else if constexpr (KIND == 5) {
#pragma unroll
            for (int k = 0; k < 8; k++)  // the clobbers make the compiler allocate a0-a7
                asm volatile("v_accvgpr_read_b32 %0, a%1" : "=v"(a[k]) : "n"(k) : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7");
        } else {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_fmac_f32_e32 %0, 0x3f7fbe77, %1" : "+v"(a[k]) : "v"(c));
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k] + p[k].x + p[k].y;
    out[blockIdx.x * 64 + threadIdx.x] = s + lds[threadIdx.x];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int iters = 2000;
    const int nwg_max = 256 * 4 * 4;
    float *out;
    long long *cyc;
    hipMalloc(&out, nwg_max * 64 * sizeof(float));
    hipMalloc(&cyc, nwg_max * sizeof(long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[7] = {"fma", "pk_fma", "dep", "dpp_add", "fmac_e32", "acc_read", "fmac_lit"};
    for (int kind = 0; kind < 7; kind++)
        for (int wps : {1, 2, 4}) {
            const int nwg = 256 * 4 * wps;
            // LDS per workgroup so that 4 * wps workgroups fit in 160 KiB per CU
            const size_t lds = (160 * 1024) / (4 * wps) - 256;
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                switch (kind) {
                    case 0: k_probe<0><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    case 1: k_probe<1><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    case 2: k_probe<2><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    case 3: k_probe<3><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    case 4: k_probe<4><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    case 5: k_probe<5><<<nwg, 64, lds>>>(out, iters, cyc); break;
                    default: k_probe<6><<<nwg, 64, lds>>>(out, iters, cyc); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            std::vector<long long> c(nwg);
            hipMemcpy(c.data(), cyc, nwg * sizeof(long long), hipMemcpyDeviceToHost);
            double avg = 0, mx = 0;
            for (auto v : c) {
                avg += v;
                mx = v > mx ? v : mx;
            }
            avg /= nwg;
            const double instrs = 8.0 * 16 * iters;
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_instr_per_wave\": %.3f, "
                   "\"max_wave\": %.3f, \"simd_cycles_per_instr\": %.3f, \"clock_ghz\": %.3f}\n",
                   names[kind], wps, ms, avg / instrs, mx / instrs, avg / instrs / wps,
                   avg / (ms * 1e-3) / 1e9);
        }
    return 0;
}
