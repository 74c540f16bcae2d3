// Policy + value heads, eval mode, one fused kernel.
//
// Replaces (network.py:102-115 + :180):
//   p = relu(policy_bn(policy_conv1x1(h)))  -> view [B,450] (channel-major, NCHW flatten)
//   logits = policy_fc(p)                    [450 -> 225]
//   probs = softmax(logits, dim=1)
//   v = relu(value_bn(value_conv1x1(h)))     -> [B,225]
//   v = relu(value_fc1(v)); value = tanh(value_fc2(v))
//
// HBM-bound: the only large read is the tower output (225*C floats per board);
// the FC weights (405 KB + 58 KB) are L2-resident and each load is reused for
// HG boards.  One 256-thread workgroup handles HG boards:
//   phase 1: one wave per (board, pixel) row: 3 dot products over C with wave
//            reductions -> folded BN + ReLU -> LDS features;
//   phase 2: thread j computes logit j for HG boards (transposed weights, coalesced);
//   phase 3: waves 0..HG-1 softmax one board each; waves HG.. run the value MLP.
#include "pv_common.h"

namespace azg {

constexpr int HG = 2;   // boards per workgroup

template <int C>
__global__ __launch_bounds__(256) void heads_fwd(
    const float* __restrict__ act,
    const float* __restrict__ wpc,    // policy_conv.weight [2][C]
    const float* __restrict__ wvc,    // value_conv.weight [C]
    const float* __restrict__ hscale, // [3] folded BN scale: policy ch0, ch1, value
    const float* __restrict__ hshift, // [3]
    const float* __restrict__ wpfT,   // policy_fc.weight^T [450][225]
    const float* __restrict__ bpf,    // [225]
    const float* __restrict__ wv1T,   // value_fc1.weight^T [225][64]
    const float* __restrict__ bv1,    // [64]
    const float* __restrict__ wv2,    // [64]
    const float* __restrict__ bv2,    // [1]
    float* __restrict__ probs, float* __restrict__ values, float* __restrict__ logits, int B)
{
    __shared__ float fp[HG][2 * PIX];
    __shared__ float fv[HG][PIX];
    __shared__ float lg[HG][ACTIONS];

    constexpr int CPL = C / 64;   // channels per lane
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b0 = blockIdx.x * HG;

    float w0[CPL], w1[CPL], w2[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        w0[q] = wpc[lane * CPL + q];
        w1[q] = wpc[C + lane * CPL + q];
        w2[q] = wvc[lane * CPL + q];
    }
    const float s0 = hscale[0], s1 = hscale[1], s2 = hscale[2];
    const float t0 = hshift[0], t1 = hshift[1], t2 = hshift[2];

    for (int task = wid; task < HG * PIX; task += 4) {
        const int g = task / PIX, p = task - g * PIX;
        const int b = b0 + g;
        if (b >= B) break;
        const float* row = act + pad_off(b * PIX + p, C) + lane * CPL;
        float d0 = 0.f, d1 = 0.f, d2 = 0.f;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            const float a = row[q];
            d0 = fmaf(a, w0[q], d0);
            d1 = fmaf(a, w1[q], d1);
            d2 = fmaf(a, w2[q], d2);
        }
        d0 = wave_sum(d0);
        d1 = wave_sum(d1);
        d2 = wave_sum(d2);
        if (lane == 0) {
            fp[g][p] = fmaxf(d0 * s0 + t0, 0.f);
            fp[g][PIX + p] = fmaxf(d1 * s1 + t1, 0.f);
            fv[g][p] = fmaxf(d2 * s2 + t2, 0.f);
        }
    }
    __syncthreads();

    if (tid < ACTIONS) {
        float acc[HG];
#pragma unroll
        for (int g = 0; g < HG; ++g) acc[g] = 0.f;
        for (int k = 0; k < 2 * PIX; ++k) {
            const float w = wpfT[k * ACTIONS + tid];
#pragma unroll
            for (int g = 0; g < HG; ++g) acc[g] = fmaf(w, fp[g][k], acc[g]);
        }
        const float bias = bpf[tid];
#pragma unroll
        for (int g = 0; g < HG; ++g) {
            const float l = acc[g] + bias;
            lg[g][tid] = l;
            if (logits && b0 + g < B) logits[(size_t)(b0 + g) * ACTIONS + tid] = l;
        }
    }
    __syncthreads();

    if (wid < HG) {
        const int g = wid, b = b0 + g;
        if (b < B) {
            float mx = -INFINITY;
            for (int j = lane; j < ACTIONS; j += 64) mx = fmaxf(mx, lg[g][j]);
            mx = wave_max(mx);
            float e[4];
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = lane + 64 * q;
                e[q] = j < ACTIONS ? expf(lg[g][j] - mx) : 0.f;
                sum += e[q];
            }
            sum = wave_sum(sum);
            const float inv = 1.f / sum;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = lane + 64 * q;
                if (j < ACTIONS) probs[(size_t)b * ACTIONS + j] = e[q] * inv;
            }
        }
    } else if (wid < 2 * HG) {
        const int g = wid - HG, b = b0 + g;
        if (b < B) {
            float hsum = bv1[lane];
            for (int k = 0; k < PIX; ++k) hsum = fmaf(wv1T[k * VHID + lane], fv[g][k], hsum);
            hsum = fmaxf(hsum, 0.f);
            float v = wave_sum(hsum * wv2[lane]) + bv2[0];
            if (lane == 0) values[b] = tanhf(v);
        }
    }
}

hipError_t launch_heads_fwd(int C, const float* act, const float* wpc, const float* wvc,
                            const float* hscale, const float* hshift, const float* wpfT,
                            const float* bpf, const float* wv1T, const float* bv1,
                            const float* wv2, const float* bv2, float* probs, float* values,
                            float* logits, int B, hipStream_t st)
{
    dim3 grid((B + HG - 1) / HG);
#define AZG_HEADS_CASE(CC)                                                                       \
    case CC:                                                                                     \
        hipLaunchKernelGGL((heads_fwd<CC>), grid, dim3(256), 0, st, act, wpc, wvc, hscale, hshift, \
                           wpfT, bpf, wv1T, bv1, wv2, bv2, probs, values, logits, B);          \
        return hipGetLastError();
    switch (C) {
        AZG_HEADS_CASE(64)
        AZG_HEADS_CASE(128)
        AZG_HEADS_CASE(256)
        default: return hipErrorInvalidValue;
    }
#undef AZG_HEADS_CASE
}

}  // namespace azg
