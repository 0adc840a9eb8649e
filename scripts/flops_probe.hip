// Calibration of gfx950's SQ_INSTS_VALU_FLOPS_FP32 counter (round 6, VERDICT
// r05 item 5): does it count the packed v_pk_{fma,mul,add}_f32 the PGS loops
// issue, and with what weight?  Each kernel runs one 64-lane wave through
// N = 4096 instructions of one kind (inline asm, so the instruction is exactly
// the one named), then one vector store.  Run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 \
//     SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 -- scripts/bin/flops_probe
// and divide each kernel's counts by N (scripts/flops_probe.sh).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int N = 4096;

#define PROBE(NAME, ASM)                                                          \
    __global__ void NAME(float *out) {                                          \
        float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f, d = 0.25f;        \
        _Pragma("unroll 64") for (int i = 0; i < N; i++) asm volatile(ASM      \
                                                                      : "+v"(a), "+v"(d) \
                                                                      : "v"(b), "v"(c)); \
        out[blockIdx.x * 64 + threadIdx.x] = a + d;                              \
    }

PROBE(k_fma_f32, "v_fma_f32 %0, %0, %2, %3")
PROBE(k_mul_f32, "v_mul_f32 %0, %0, %2")
PROBE(k_add_f32, "v_add_f32 %0, %0, %2")
// packed: a/d as a register pair would need a 64-bit operand; use one
// 64-bit asm operand instead
#define PROBE2(NAME, ASM)                                                        \
    __global__ void NAME(float *out) {                                          \
        typedef float f2 __attribute__((ext_vector_type(2)));                    \
        f2 a = {threadIdx.x * 1e-3f, 0.5f}, b = {1.0001f, 0.9999f}, c = {0.5f, 0.25f}; \
        _Pragma("unroll 64") for (int i = 0; i < N; i++) asm volatile(ASM : "+v"(a) : "v"(b), "v"(c)); \
        out[blockIdx.x * 64 + threadIdx.x] = a.x + a.y;                          \
    }
PROBE2(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %2")
PROBE2(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
PROBE2(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")

int main() {
    float *out;
    if (hipMalloc(&out, 64 * sizeof(float)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_fma_f32, dim3(1), dim3(64), 0, 0, out);
    hipLaunchKernelGGL(k_mul_f32, dim3(1), dim3(64), 0, 0, out);
    hipLaunchKernelGGL(k_add_f32, dim3(1), dim3(64), 0, 0, out);
    hipLaunchKernelGGL(k_pk_fma_f32, dim3(1), dim3(64), 0, 0, out);
    hipLaunchKernelGGL(k_pk_mul_f32, dim3(1), dim3(64), 0, 0, out);
    hipLaunchKernelGGL(k_pk_add_f32, dim3(1), dim3(64), 0, 0, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    float h[64];
    if (hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("flops_probe done (N = %d per kernel, one wave each): %g\n", N, h[0]);
    (void)hipFree(out);
    return 0;
}
