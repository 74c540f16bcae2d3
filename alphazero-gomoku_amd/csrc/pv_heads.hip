// Policy + value heads (network.py:102-115 + softmax at :180), two kernels.
//
//   heads_project<C, BN>: the three 1x1 projections of the tower output
//       (policy_conv C->2, value_conv C->1) for every pixel, optionally followed
//       by the folded eval BatchNorm + ReLU; writes h[b][3][225] (channel-major,
//       i.e. exactly the NCHW flatten order network.py:105,112 uses).  HBM-bound:
//       reads 225*C*4 B per board once; 4 consecutive threads cover one pixel's
//       C channels (coalesced 128-B quarter rows), partial dots reduced by 2 xor
//       shuffles.  Also used raw (BN = false) by the train step.
//   small_gemm (pv_gemm.hip) + heads_finalize: policy_fc 450->225 and value_fc1
//       225->64 as one two-problem fp32-MFMA GEMM launch, then bias, softmax, ReLU,
//       value_fc2 64->1 and tanh, one wave per board.
#include "pv_internal.h"

namespace azg {

constexpr int PROJ_ROWS = 64;   // pixels per workgroup in heads_project

template <int C, bool BN>
__global__ __launch_bounds__(256) void heads_project(const float* __restrict__ act, const float* __restrict__ wpc,
                                                     const float* __restrict__ wvc,
                                                     const float* __restrict__ hscale,
                                                     const float* __restrict__ hshift, float* __restrict__ hout,
                                                     int M, int fs, int voff)
{
    constexpr int Q = C / 4;        // channels per thread
    __shared__ float w[3][C];
    for (int i = threadIdx.x; i < 3 * C; i += 256) w[i / C][i % C] = i < 2 * C ? wpc[i] : wvc[i - 2 * C];
    __syncthreads();
    const int q = threadIdx.x & 3;
    const int m = blockIdx.x * PROJ_ROWS + (threadIdx.x >> 2);
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    if (m < M) {
        const float* row = act + pad_off(m, C) + q * Q;
#pragma unroll
        for (int c = 0; c < Q; c += 4) {
            const f32x4 a = *(const f32x4*)(row + c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                d0 = fmaf(a[k], w[0][q * Q + c + k], d0);
                d1 = fmaf(a[k], w[1][q * Q + c + k], d1);
                d2 = fmaf(a[k], w[2][q * Q + c + k], d2);
            }
        }
    }
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) {
        d0 += __shfl_xor(d0, o, 64);
        d1 += __shfl_xor(d1, o, 64);
        d2 += __shfl_xor(d2, o, 64);
    }
    if (m < M && q == 0) {
        const int b = m / PIX, p = m - b * PIX;
        float* hb = hout + (size_t)b * fs;
        if (BN) {
            d0 = head_bn_relu(d0, hscale[0], hshift[0]);
            d1 = head_bn_relu(d1, hscale[1], hshift[1]);
            d2 = head_bn_relu(d2, hscale[2], hshift[2]);
        }
        hb[p] = d0;
        hb[PIX + p] = d1;
        hb[voff + p] = d2;
    }
}

// policy_fc + value_fc1 (network.py:104-106, 112-114) on fp32 MFMA: one workgroup
// per 32 boards x 32 outputs (grid.y: 8 policy tiles then 2 value tiles, rows of
// the packed wfc), K split over the 4 waves in blocks of 8: lane (r, h) loads one
// float4 of its board's features and one float4 of its output's weights per block
// (k = 8q + 4h + t, t = MFMA step), all loads of a wave issued before its first
// MFMA; partial tiles summed in fixed wave order.  Each output row depends only on
// its own board (batch independent).
__global__ __launch_bounds__(256) void heads_fc(const float* __restrict__ feat, const float* __restrict__ wfc,
                                                float* __restrict__ pre, int B)
{
    constexpr int QMAX = (FC_KP / 8 + 3) / 4;    // blocks per wave, at most
    __shared__ float red[4][16][64];
    const int tile = blockIdx.y;
    const bool val = tile >= 8;
    const int j0 = val ? ACTIONS + (tile - 8) * 32 : tile * 32;   // first output (= wfc row)
    const int koff = val ? FC_KP : 0;
    const int nblk = (val ? FC_KV : FC_KP) / 8;
    const int i0 = blockIdx.x * 32;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    const float* a = feat + (size_t)min(i0 + r32, B - 1) * FC_FS + koff + 4 * h;
    const float* w = wfc + (size_t)min(j0 + r32, FC_OUT - 1) * FC_KP + 4 * h;
    const int q0 = wid * nblk / 4, nq = (wid + 1) * nblk / 4 - q0;
    f32x4 av[QMAX], bv[QMAX];
#pragma unroll
    for (int u = 0; u < QMAX; ++u)
        if (u < nq) {
            av[u] = *(const f32x4*)(a + (q0 + u) * 8);
            bv[u] = *(const f32x4*)(w + (q0 + u) * 8);
        }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int u = 0; u < QMAX; ++u)
        if (u < nq) {
#pragma unroll
            for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][t], bv[u][t], acc, 0, 0, 0);
        }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wid][r][lane] = acc[r];
    __syncthreads();
    if (wid == 0) {
        const int j = j0 + r32;
        const bool jok = val || j < ACTIONS;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = ((red[0][r][lane] + red[1][r][lane]) + red[2][r][lane]) + red[3][r][lane];
            const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (i < B && jok) pre[(size_t)i * FC_OUT + j] = v;
        }
    }
}

// Per board (one wave): logits = pre + bias, softmax; value = tanh(relu(pre_v + b1) . w2 + b2).
// priors (optional, with boards): probs * (board == 0), the reference's masked
// prior p * valid (mcts/new_mcts_alpha.py:166) -- float32 multiply by 1.0 / 0.0.
__global__ __launch_bounds__(256) void heads_finalize(const float* __restrict__ pre, const float* __restrict__ bpf,
                                                      const float* __restrict__ bv1, const float* __restrict__ wv2,
                                                      const float* __restrict__ bv2, float* __restrict__ probs,
                                                      float* __restrict__ values, float* __restrict__ logits, int B,
                                                      const int8_t* __restrict__ boards, float* __restrict__ priors)
{
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const float* pb = pre + (size_t)b * FC_OUT;
    float lg[4];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        lg[t] = j < ACTIONS ? pb[j] + bpf[j] : -INFINITY;
        mx = fmaxf(mx, lg[t]);
    }
    mx = wave_max(mx);
    float e[4], sum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        e[t] = j < ACTIONS ? expf(lg[t] - mx) : 0.f;
        sum += e[t];
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        if (j < ACTIONS) {
            const float pj = e[t] * inv;
            probs[(size_t)b * ACTIONS + j] = pj;
            if (logits) logits[(size_t)b * ACTIONS + j] = lg[t];
            if (priors) priors[(size_t)b * ACTIONS + j] = pj * (boards[(size_t)b * PIX + j] == 0 ? 1.f : 0.f);
        }
    }
    const float hid = fmaxf(pb[ACTIONS + lane] + bv1[lane], 0.f);
    const float v = wave_sum(hid * wv2[lane]) + bv2[0];
    if (lane == 0) values[b] = tanhf(v);
}

hipError_t launch_heads_project(int C, bool bn, const float* act, const float* wpc, const float* wvc,
                                const float* hscale, const float* hshift, float* hout, int M, hipStream_t st,
                                int fs, int voff)
{
    dim3 grid((M + PROJ_ROWS - 1) / PROJ_ROWS);
#define AZG_PROJ_CASE(CC)                                                                                      \
    case CC:                                                                                                   \
        if (bn) hipLaunchKernelGGL((heads_project<CC, true>), grid, dim3(256), 0, st, act, wpc, wvc, hscale, hshift, hout, M, fs, voff); \
        else hipLaunchKernelGGL((heads_project<CC, false>), grid, dim3(256), 0, st, act, wpc, wvc, hscale, hshift, hout, M, fs, voff); \
        return hipGetLastError();
    switch (C) {
        AZG_PROJ_CASE(64)
        AZG_PROJ_CASE(128)
        AZG_PROJ_CASE(256)
        default: return hipErrorInvalidValue;
    }
#undef AZG_PROJ_CASE
}

// the fc forward alone (train step, key 28 bit 3): feat [B][FC_FS] -> pre [B][FC_OUT]
hipError_t launch_heads_fc(const float* feat, const float* wfc, float* pre, int B, hipStream_t st)
{
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(heads_fc, dim3((B + 31) / 32, 10), dim3(256), 0, st, feat, wfc, pre, B);
    return hipGetLastError();
}

hipError_t launch_heads_fwd(int C, const float* act, const float* wpc, const float* wvc, const float* hscale,
                            const float* hshift, const float* wfc, const float* bpf,
                            const float* bv1, const float* wv2, const float* bv2, float* hbuf, float* probs,
                            float* values, float* logits, int B, hipStream_t st, const int8_t* boards,
                            float* priors, bool projected)
{
    if (B <= 0) return hipSuccess;
    // hbuf: [B][FC_FS] features (zero pads, set at allocation) then pre [B][FC_OUT]; the
    // board16 tower writes the features itself (projected)
    hipError_t e = projected ? hipSuccess
                             : launch_heads_project(C, true, act, wpc, wvc, hscale, hshift, hbuf, B * PIX, st, FC_FS,
                                                    FC_KP);
    if (e != hipSuccess) return e;
    float* pre = hbuf + (size_t)B * FC_FS;
    hipLaunchKernelGGL(heads_fc, dim3((B + 31) / 32, 10), dim3(256), 0, st, hbuf, wfc, pre, B);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(heads_finalize, dim3((B + 3) / 4), dim3(256), 0, st, pre, bpf, bv1, wv2, bv2, probs, values,
                       logits, B, boards, priors);
    return hipGetLastError();
}

}  // namespace azg
