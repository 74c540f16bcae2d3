// Shared definitions for the gfx950 policy/value kernels.
//
// Activation layout in HBM ("padded NHWC"): act[b][17][17][C] fp32, the 1-pixel
// zero halo is written once at allocation and never touched again, so every
// 3x3 tap of an interior pixel is an unconditional load.  Pixel m of the batch
// (m = b*225 + y*15 + x) lives at element ((b*289 + (y+1)*17 + (x+1)) * C).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace azg {

constexpr int BOARD = 15;
constexpr int PIX = BOARD * BOARD;        // 225
constexpr int PADW = BOARD + 2;           // 17
constexpr int PADPIX = PADW * PADW;       // 289
constexpr int ACTIONS = PIX;              // 225
constexpr int VHID = 64;                  // value_fc1 width (network.py:70)
// eval head features, per board (16-B aligned rows): policy planes (450, padded to
// FC_KP = 456) then the value plane (225, padded to FC_KV = 232); packed head FC
// weights wfc[FC_OUT][FC_KP]: rows 0..224 policy_fc (K = 450), 225..288 value_fc1
// (K = 225), zero-padded.  The pads are zero and never written.
constexpr int FC_KP = 456;
constexpr int FC_KV = 232;
constexpr int FC_FS = FC_KP + FC_KV;      // 688 floats per board
constexpr int FC_OUT = ACTIONS + VHID;    // 289: pre[b] = [policy logits | value hidden]
constexpr float BN_EPS = 1e-5f;           // nn.BatchNorm2d default
constexpr float BN_MOMENTUM = 0.1f;       // nn.BatchNorm2d default

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// element offset of interior pixel m in a padded NHWC tensor with C channels
__device__ __forceinline__ int pad_off(int m, int C) {
    int b = m / PIX;
    int p = m - b * PIX;
    int y = p / BOARD;
    int x = p - y * BOARD;
    return (b * PADPIX + (y + 1) * PADW + (x + 1)) * C;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Write-through (sc1) 16-B / 4-B stores through a raw buffer resource: a kernel whose
// outputs are stored this way leaves no dirty L2 lines behind, so the dependent launch
// does not wait for their write-back at the kernel boundary (MI355X_MICROARCH.md
// "boundary": + B / 6 TB/s for B dirty bytes; a train conv leaves 14.7 MB at B=128).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <bool WT>
__device__ __forceinline__ void store4(float* base, __amdgpu_buffer_rsrc_t rs, int off, f32x4 v) {
    if constexpr (WT)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                               rs, off * 4, 0, 16);
    else
        *(f32x4*)(base + off) = v;
}
template <bool WT>
__device__ __forceinline__ void store1(float* base, __amdgpu_buffer_rsrc_t rs, int off, float v) {
    if constexpr (WT)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, off * 4, 0, 16);
    else
        base[off] = v;
}
// bytes of a padded NHWC tensor holding the M interior pixels (whole boards)
__device__ __forceinline__ size_t padded_bytes(int M, int C) {
    return (size_t)((M + PIX - 1) / PIX) * PADPIX * C * sizeof(float);
}

// BatchNorm backward apply of one element (reference network.py:12-25 autograd; shared
// by bn_bwd_apply_kernel, the fused dgrad epilogue and the persistent backward):
// dy = g * (act > 0); dz = ((dy - gm) - (z - mean) * k) * iw.
__device__ __forceinline__ float bnbwd_elem(float g, float av, float z, float mu, float gm, float k, float iw,
                                            float& dy)
{
    dy = av > 0.f ? g : 0.f;
    return ((dy - gm) - (z - mu) * k) * iw;
}

enum Epi : int {
    EPI_BN_RELU = 0,      // relu(acc*scale + shift)
    EPI_BN_RES_RELU = 1,  // relu(acc*scale + shift + resid)
    EPI_RAW = 2,          // acc (train-mode conv output, dgrad)
    EPI_ADD = 3,          // acc + resid (dgrad into an existing residual gradient)
};

}  // namespace azg
