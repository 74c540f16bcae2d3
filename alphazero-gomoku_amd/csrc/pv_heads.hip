// Policy + value heads (network.py:102-115 + softmax at :180), two kernels.
//
//   heads_project<C, BN>: the three 1x1 projections of the tower output
//       (policy_conv C->2, value_conv C->1) for every pixel, optionally followed
//       by the folded eval BatchNorm + ReLU; writes h[b][3][225] (channel-major,
//       i.e. exactly the NCHW flatten order network.py:105,112 uses).  HBM-bound:
//       reads 225*C*4 B per board once; 4 consecutive threads cover one pixel's
//       C channels (coalesced 128-B quarter rows), partial dots reduced by 2 xor
//       shuffles.  Also used raw (BN = false) by the train step.
//   heads_fc_eval: per workgroup HB boards: policy_fc 450->225 (+bias), softmax,
//       value_fc1 225->64 + ReLU, value_fc2 64->1, tanh.  Each transposed weight
//       load (coalesced, L2-resident) is reused for HB boards.
#include "pv_internal.h"

namespace azg {

constexpr int PROJ_ROWS = 64;   // pixels per workgroup in heads_project
constexpr int HB = 8;           // boards per workgroup in heads_fc_eval

template <int C, bool BN>
__global__ __launch_bounds__(256) void heads_project(const float* __restrict__ act, const float* __restrict__ wpc,
                                                     const float* __restrict__ wvc,
                                                     const float* __restrict__ hscale,
                                                     const float* __restrict__ hshift, float* __restrict__ hout,
                                                     int M)
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
        float* hb = hout + (size_t)b * 3 * PIX;
        if (BN) {
            d0 = fmaxf(d0 * hscale[0] + hshift[0], 0.f);
            d1 = fmaxf(d1 * hscale[1] + hshift[1], 0.f);
            d2 = fmaxf(d2 * hscale[2] + hshift[2], 0.f);
        }
        hb[p] = d0;
        hb[PIX + p] = d1;
        hb[2 * PIX + p] = d2;
    }
}

__global__ __launch_bounds__(256) void heads_fc_eval(
    const float* __restrict__ feat,   // [B][3*225]: policy features 0..449, value features 450..674
    const float* __restrict__ wpfT,   // policy_fc.weight^T [450][225]
    const float* __restrict__ bpf,    // [225]
    const float* __restrict__ wv1T,   // value_fc1.weight^T [225][64]
    const float* __restrict__ bv1,    // [64]
    const float* __restrict__ wv2,    // [64]
    const float* __restrict__ bv2,    // [1]
    float* __restrict__ probs, float* __restrict__ values, float* __restrict__ logits, int B)
{
    __shared__ float f[HB][3 * PIX];
    __shared__ float lg[HB][ACTIONS];
    __shared__ float hid[HB][VHID];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b0 = blockIdx.x * HB;
    const int nb = min(HB, B - b0);
    for (int i = tid; i < HB * 3 * PIX; i += 256) {
        const int g = i / (3 * PIX);
        f[g][i - g * 3 * PIX] = g < nb ? feat[(size_t)b0 * 3 * PIX + i] : 0.f;
    }
    __syncthreads();
    if (tid < ACTIONS) {
        float acc[HB];
#pragma unroll
        for (int g = 0; g < HB; ++g) acc[g] = 0.f;
#pragma unroll 4
        for (int k = 0; k < 2 * PIX; ++k) {
            const float wk = wpfT[k * ACTIONS + tid];
#pragma unroll
            for (int g = 0; g < HB; ++g) acc[g] = fmaf(wk, f[g][k], acc[g]);
        }
        const float bias = bpf[tid];
#pragma unroll
        for (int g = 0; g < HB; ++g) lg[g][tid] = acc[g] + bias;
    }
    {
        // value hidden layer: thread -> unit i = tid % 64, boards (tid / 64) + 4 j
        const int i = tid & 63, gq = tid >> 6;
        constexpr int GPT = HB / 4;
        float acc[GPT];
#pragma unroll
        for (int j = 0; j < GPT; ++j) acc[j] = 0.f;
#pragma unroll 4
        for (int k = 0; k < PIX; ++k) {
            const float wk = wv1T[k * VHID + i];
#pragma unroll
            for (int j = 0; j < GPT; ++j) acc[j] = fmaf(wk, f[gq + 4 * j][2 * PIX + k], acc[j]);
        }
#pragma unroll
        for (int j = 0; j < GPT; ++j) hid[gq + 4 * j][i] = fmaxf(acc[j] + bv1[i], 0.f);
    }
    __syncthreads();
    // softmax + value: wave w handles boards w, w+4, ...
    for (int g = wid; g < nb; g += 4) {
        const int b = b0 + g;
        float mx = -INFINITY;
        for (int j = lane; j < ACTIONS; j += 64) mx = fmaxf(mx, lg[g][j]);
        mx = wave_max(mx);
        float e[4];
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = lane + 64 * t;
            e[t] = j < ACTIONS ? expf(lg[g][j] - mx) : 0.f;
            sum += e[t];
        }
        sum = wave_sum(sum);
        const float inv = 1.f / sum;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = lane + 64 * t;
            if (j < ACTIONS) {
                probs[(size_t)b * ACTIONS + j] = e[t] * inv;
                if (logits) logits[(size_t)b * ACTIONS + j] = lg[g][j];
            }
        }
        const float v = wave_sum(hid[g][lane] * wv2[lane]) + bv2[0];
        if (lane == 0) values[b] = tanhf(v);
    }
}

hipError_t launch_heads_project(int C, bool bn, const float* act, const float* wpc, const float* wvc,
                                const float* hscale, const float* hshift, float* hout, int M, hipStream_t st)
{
    dim3 grid((M + PROJ_ROWS - 1) / PROJ_ROWS);
#define AZG_PROJ_CASE(CC)                                                                                      \
    case CC:                                                                                                   \
        if (bn) hipLaunchKernelGGL((heads_project<CC, true>), grid, dim3(256), 0, st, act, wpc, wvc, hscale, hshift, hout, M); \
        else hipLaunchKernelGGL((heads_project<CC, false>), grid, dim3(256), 0, st, act, wpc, wvc, hscale, hshift, hout, M); \
        return hipGetLastError();
    switch (C) {
        AZG_PROJ_CASE(64)
        AZG_PROJ_CASE(128)
        AZG_PROJ_CASE(256)
        default: return hipErrorInvalidValue;
    }
#undef AZG_PROJ_CASE
}

hipError_t launch_heads_fwd(int C, const float* act, const float* wpc, const float* wvc, const float* hscale,
                            const float* hshift, const float* wpfT, const float* bpf, const float* wv1T,
                            const float* bv1, const float* wv2, const float* bv2, float* hbuf, float* probs,
                            float* values, float* logits, int B, hipStream_t st)
{
    hipError_t e = launch_heads_project(C, true, act, wpc, wvc, hscale, hshift, hbuf, B * PIX, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(heads_fc_eval, dim3((B + HB - 1) / HB), dim3(256), 0, st, hbuf, wpfT, bpf, wv1T, bv1, wv2,
                       bv2, probs, values, logits, B);
    return hipGetLastError();
}

}  // namespace azg
