// Microbenchmark: sustained FLOP/s of v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16
// chains (operands in registers, random data, 4 waves per SIMD, every CU busy): how much
// of the chip's clock each MFMA shape keeps under full load (MI355X_MICROARCH.md DVFS).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k32(const f16x8* in, float* out, int iters)
{
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f32x16 c0 = {}, c1 = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k16(const f16x8* in, float* out, int iters)
{
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {   // 4 x 16x16x32 = the FLOPs of 2 x 32x32x16 ... x2
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, b, c3, 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main()
{
    std::vector<_Float16> h(512 * 8);
    unsigned x = 1;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (_Float16)(((x >> 9) & 1023) / 1024.f - 0.5f); }
    f16x8* din; float* dout;
    hipMalloc(&din, h.size() * 2); hipMalloc(&dout, 256 * 4 * 1024 * 4);
    hipMemcpy(din, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const int blocks = 256 * 4, iters = 4000;   // 4 workgroups of 4 waves per CU = 4 waves per SIMD
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep)
        for (int which = 0; which < 2; ++which) {
            float ms;
            hipEventRecord(e0);
            for (int t = 0; t < 5; ++t) {
                if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
            }
            hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
            // k32: 16 MFMA 32x32x16 per iter = 16 * 32768 FLOP; k16: 32 MFMA 16x16x32 = 32 * 16384
            const double flop = 5.0 * blocks * 4.0 * iters * 16 * 32768;
            printf("%s: %.1f TFLOP/s\n", which == 0 ? "32x32x16" : "16x16x32", flop / (ms * 1e-3) / 1e12);
        }
    return 0;
}
