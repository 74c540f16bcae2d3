// Train-step head chain (reference network.py:101-115 forward in train mode, the
// loss of network.py:216-221 and its backward down to the tower output), as short,
// wide launches (the chain is latency-bound: every launch here is 6-16 us):
//
//   head_proj_stats_kernel  the last block's BN2 + residual + ReLU (the tower output
//       a = relu(z*s + t + x), written for the backward) fused with the three 1x1
//       head projections (policy_conv C->2, value_conv C->1: zh[b][3][225]) and
//       per-workgroup fp64 partials of the head BatchNorms' batch statistics;
//   head_bn_apply_feat_kernel  every workgroup finalizes the head statistics from those
//       partials in one fixed order (workgroup 0 publishes mean / invstd / scale / shift,
//       the running stats and every BN layer's num_batches_tracked += 1), then head BN +
//       ReLU into fp / fv and the eval forward's padded feature rows for heads_fc;
//   heads_fc (pv_heads.hip) + heads_loss_kernel (pv_train.hip): the fc forward, log_softmax
//       + KLDiv(batchmean) + MSE and their gradients;
//   head_dgrad_kernel  the masked fc data gradients dfp / dfv (fp32 MFMA) with per-
//       workgroup head-BN backward partials;
//   heads_bwd_fused_kernel  every workgroup finalizes the head-BN backward from those
//       partials (workgroup 0 publishes dgamma / dbeta), applies it per pixel on the fly,
//       and writes the projections' data gradient gX = sum_ch dzh * Wh, their weight-grad
//       partials, and the BatchNorm-backward partial sums of the last block's bn2 (dy =
//       gX * (a > 0), S dy, S (z - mean) dy per 128-row tile) for the tower backward.
//
// The fc weight gradients (dW = dlogits^T fp, dW1 = dhv^T fv, head_fc_wgrad_kernel) run
// at the end of the step, off the critical path.
#include "pv_train_heads.h"

#include <type_traits>

namespace azg {

constexpr int HP_ROWS = 64;     // pixels per workgroup of head_proj_stats_kernel
__device__ __forceinline__ void st_wt_d(double* p, double v)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v),
                                          wt_rsrc(p, 8), 0, 0, 16);
}
__device__ __forceinline__ double wsum_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// finalize of the head BN statistics from nwg per-workgroup fp64 partials [nwg][6]:
// thread t sums workgroups t, t + 256, ... (all loads issued first), then a fixed-order
// block reduction (256 threads; red: [4][6]); shared by the last-arriving workgroup of
// head_proj_stats_kernel and the one-workgroup head_proj_fin_kernel (bitwise equal)
// coef (LDS, optional): the folded scale / shift of the three channels for the caller's
// own use; write: publish mean / invstd / scale / shift, the running stats and the
// num_batches_tracked increments (exactly one workgroup per step may write)
__device__ __forceinline__ void head_stats_fin(const HeadStatsArgs& a, int nwg, double (*red)[6],
                                               float* coef = nullptr, bool write = true)
{
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double s[6] = {0, 0, 0, 0, 0, 0};
    for (int g0 = threadIdx.x; g0 < nwg; g0 += 512) {
        double x0[6], x1[6];
        const bool two = g0 + 256 < nwg;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            x0[k] = a.part[(size_t)g0 * 6 + k];
            x1[k] = two ? a.part[(size_t)(g0 + 256) * 6 + k] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) s[k] += x0[k] + x1[k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = wsum_d(s[k]);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) red[wid][k] = s[k];
    __syncthreads();
    if (wid == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) s[k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
        if (lane < 3) {   // = head_stats_finalize_kernel
            const int ch = lane;
            const BnDesc d = a.desc[ch < 2 ? a.pol_layer : a.val_layer];
            const int c = ch < 2 ? ch : 0;
            const double N = (double)a.M;
            const double sm = ch == 0 ? s[0] : ch == 1 ? s[2] : s[4];
            const double sq = ch == 0 ? s[1] : ch == 1 ? s[3] : s[5];
            const double mean = sm / N;
            double qv = sq - sm * mean;
            qv = qv > 0.0 ? qv : 0.0;
            const double var = qv / N;
            const float mean_f = (float)mean;
            const float inv_f = (float)(1.0 / sqrt(var + (double)BN_EPS));
            const float alpha = inv_f * a.params[d.gamma_off + c];
            const float shift = a.params[d.beta_off + c] - mean_f * alpha;
            if (coef) {
                coef[ch] = alpha;
                coef[3 + ch] = shift;
            }
            if (write) {
                a.bmean[d.out_off + c] = mean_f;
                a.binv[d.out_off + c] = inv_f;
                a.bscale[d.out_off + c] = alpha;
                a.bshift[d.out_off + c] = shift;
                const double unb = N > 1 ? qv / (N - 1.0) : var;
                float* rm = a.stats + d.stat_off;
                float* rv = a.stats + d.stat_off + d.c;
                rm[c] = (float)((double)BN_MOMENTUM * mean + (1.0 - (double)BN_MOMENTUM) * (double)rm[c]);
                rv[c] = (float)((double)BN_MOMENTUM * unb + (1.0 - (double)BN_MOMENTUM) * (double)rv[c]);
            }
        }
    }
    if (write && a.nbt)
        for (int i = threadIdx.x; i < a.nbn; i += 256) a.nbt[i] += 1;
}
// partials only: every workgroup of head_bn_apply_feat_kernel finalizes them
template <int C, bool APPLY>
__global__ __launch_bounds__(256) void head_proj_stats_kernel(const HeadStatsArgs a)
{
    // C/4 consecutive threads own one pixel (4 channels each: 16-B runs, every wave
    // instruction reads whole 128-B lines), 256*4/C pixels per pass; every load of the
    // workgroup's 64 rows is issued before the first store (the stores may alias them)
    constexpr int TPP = C / 4, PPP = 256 / TPP, NP = HP_ROWS / PPP;
    static_assert(TPP <= 64 && 64 % TPP == 0 && HP_ROWS % PPP == 0, "pixel layout");
    __shared__ double red[4][6];
    const int tid = threadIdx.x;
    const int c = (tid % TPP) * 4, pp = tid / TPP;
    const f32x4 w0 = *(const f32x4*)(a.wpc + c), w1 = *(const f32x4*)(a.wpc + C + c), w2 = *(const f32x4*)(a.wvc + c);
    f32x4 s4 = {1.f, 1.f, 1.f, 1.f}, t4 = {0.f, 0.f, 0.f, 0.f};
    if (APPLY) {
        s4 = *(const f32x4*)(a.scale + c);
        t4 = *(const f32x4*)(a.shift + c);
    }
    const int mb = blockIdx.x * HP_ROWS;
    f32x4 zv[NP], rv[APPLY ? NP : 1];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int m = mb + pp + p * PPP;
        zv[p] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (APPLY) rv[p] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m < a.M) {
            const int o = pad_off(m, C) + c;
            zv[p] = *(const f32x4*)(a.z + o);
            if (APPLY) rv[p] = *(const f32x4*)(a.res + o);
        }
    }
    const __amdgpu_buffer_rsrc_t ars = wt_rsrc(a.aout, padded_bytes(a.M, C));
    double v[6] = {0, 0, 0, 0, 0, 0};   // S z, S z^2 of the three head channels (owner lanes)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int m = mb + pp + p * PPP;
        f32x4 x = zv[p];
        if (APPLY) {   // = bn_apply_kernel<C, true>: relu(fma(z, scale, shift) + res)
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = fmaxf(fmaf(x[k], s4[k], t4[k]) + rv[p][k], 0.f);
            if (m < a.M) store4<true>(a.aout, ars, pad_off(m, C) + c, x);
        }
        float d0 = 0.f, d1 = 0.f, d2 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            d0 = fmaf(x[k], w0[k], d0);
            d1 = fmaf(x[k], w1[k], d1);
            d2 = fmaf(x[k], w2[k], d2);
        }
#pragma unroll
        for (int o = 1; o < TPP; o <<= 1) {
            d0 += __shfl_xor(d0, o, 64);
            d1 += __shfl_xor(d1, o, 64);
            d2 += __shfl_xor(d2, o, 64);
        }
        if (tid % TPP == 0 && m < a.M) {
            const int b = m / PIX, px = m - b * PIX;
            float* hb = a.zh + (size_t)b * 3 * PIX;
            hb[px] = d0;
            hb[PIX + px] = d1;
            hb[2 * PIX + px] = d2;
            v[0] += (double)d0;
            v[1] += (double)d0 * d0;
            v[2] += (double)d1;
            v[3] += (double)d1 * d1;
            v[4] += (double)d2;
            v[5] += (double)d2 * d2;
        }
    }
    // per-workgroup fp64 sums S z, S z^2 of the three head channels
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = wsum_d(v[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) red[wid][k] = v[k];
    __syncthreads();
    if (threadIdx.x < 6)
        st_wt_d(a.part + (size_t)blockIdx.x * 6 + threadIdx.x,
                (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]));
}

// = head_bn_bwd_apply_kernel (dzh on the fly) + heads_bwd_proj_kernel, and the last
// block's bn_bwd_reduce partials per 128-row tile (HROWS), same thread layout as
// heads_bwd_proj_kernel: float4 over channels, RG row groups, UNR rows in flight
__device__ __forceinline__ void head_bwd_fin_wave(const HeadDgradArgs& a, int nwg, float* hk, bool write);

template <int C, bool BNX>
__global__ __launch_bounds__(256) void heads_bwd_fused_kernel(const HeadBwdArgs a)
{
    constexpr int HROWS = 128;
    constexpr int Q = C / 4, RG = 256 / Q, UNR = 4;
    __shared__ f32x4 red[5][RG][Q];
    const int q = threadIdx.x % Q, rg = threadIdx.x / Q;
    const int c = 4 * q;
    const int m0 = blockIdx.x * HROWS;
    const int rows = min(HROWS, a.M - m0);
    const f32x4 w0 = *(const f32x4*)(a.wpc + c), w1 = *(const f32x4*)(a.wpc + C + c), w2 = *(const f32x4*)(a.wvc + c);
    f32x4 mu2 = {0.f, 0.f, 0.f, 0.f};
    if (BNX) mu2 = *(const f32x4*)(a.mean2 + c);
    // head-BN backward coefficients, finalized here by every workgroup from
    // head_dgrad_kernel's partials (one wave, fixed order; workgroup 0 publishes dgamma /
    // dbeta): the same values in every workgroup, bitwise
    __shared__ float shk[9];
    const float* hbp = a.dg.hb;
    if (a.dg_nwg) {
        if (threadIdx.x < 64) head_bwd_fin_wave(a.dg, a.dg_nwg, shk, blockIdx.x == 0);
        __syncthreads();
        hbp = shk;
    }
    float hm[3], hk[3][3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        hm[ch] = a.hmean[ch];
#pragma unroll
        for (int k = 0; k < 3; ++k) hk[ch][k] = hbp[ch * 3 + k];
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, xa = s0, xb = s0;
    for (int r0 = rg; r0 < rows; r0 += RG * UNR) {
        f32x4 xv[UNR], zv[UNR];
        float d0[UNR], d1[UNR], d2[UNR];
        int o[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int r = r0 + RG * u;
            const int m = m0 + min(r, rows - 1);
            const int b = m / PIX, p = m - b * PIX;
            const float* zb = a.zh + (size_t)b * 3 * PIX;
            const float y0 = a.dfp[(size_t)b * 2 * PIX + p], y1 = a.dfp[(size_t)b * 2 * PIX + PIX + p];
            const float y2 = a.dfv[(size_t)b * PIX + p];
            d0[u] = ((y0 - hk[0][0]) - (zb[p] - hm[0]) * hk[0][1]) * hk[0][2];
            d1[u] = ((y1 - hk[1][0]) - (zb[PIX + p] - hm[1]) * hk[1][1]) * hk[1][2];
            d2[u] = ((y2 - hk[2][0]) - (zb[2 * PIX + p] - hm[2]) * hk[2][1]) * hk[2][2];
            o[u] = pad_off(m, C) + c;
            xv[u] = *(const f32x4*)(a.act + o[u]);
            if (BNX) zv[u] = *(const f32x4*)(a.z2 + o[u]);
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (r0 + RG * u < rows) {
                f32x4 g;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    s0[e] = fmaf(d0[u], xv[u][e], s0[e]);
                    s1[e] = fmaf(d1[u], xv[u][e], s1[e]);
                    s2[e] = fmaf(d2[u], xv[u][e], s2[e]);
                    g[e] = d0[u] * w0[e] + d1[u] * w1[e] + d2[u] * w2[e];
                    if (BNX) {   // = bn_bwd_reduce_kernel: dy = g * (act > 0)
                        const float dy = xv[u][e] > 0.f ? g[e] : 0.f;
                        xa[e] += dy;
                        xb[e] = fmaf(zv[u][e] - mu2[e], dy, xb[e]);
                    }
                }
                *(f32x4*)(a.gx + o[u]) = g;
            }
        }
    }
    red[0][rg][q] = s0;
    red[1][rg][q] = s1;
    red[2][rg][q] = s2;
    red[3][rg][q] = xa;
    red[4][rg][q] = xb;
    __syncthreads();
    if (rg == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (!BNX && k >= 3) break;
            f32x4 v = red[k][0][q];
            for (int g = 1; g < RG; ++g) v += red[k][g][q];
            if (k < 3) *(f32x4*)(a.hpart + ((size_t)blockIdx.x * 3 + k) * C + c) = v;
            else *(f32x4*)((k == 3 ? a.pa : a.pb) + (size_t)blockIdx.x * C + c) = v;
        }
    }
}

// head BN + ReLU (fp, fv), also writing the features in the eval forward's padded row
// layout feat[b][FC_FS] (policy 450 -> FC_KP, value 225 at FC_KP; the zero pads are set
// at allocation) so the fc forward runs on heads_fc's 16-B operand loads
// The head BN statistics are finalized by every workgroup from head_proj_stats_kernel's
// nwg partials (one fixed-order reduction: the same coefficients in every workgroup);
// workgroup 0 publishes them with the running stats
__global__ __launch_bounds__(256) void head_bn_apply_feat_kernel(const float* __restrict__ zh,
                                                                 float* __restrict__ fp, float* __restrict__ fv,
                                                                 float* __restrict__ feat, int B,
                                                                 const HeadStatsArgs fa, int nwg)
{
    __shared__ double red[4][6];
    __shared__ float coef[6];
    head_stats_fin(fa, nwg, red, coef, blockIdx.x == 0);
    __syncthreads();
    const float* hscale = coef;
    const float* hshift = coef + 3;
    const int total = B * 3 * PIX;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int b = i / (3 * PIX), k = i - b * 3 * PIX;
        const int ch = k / PIX;
        const float y = fmaxf(zh[i] * hscale[ch] + hshift[ch], 0.f);
        if (ch < 2) {
            fp[(size_t)b * 2 * PIX + k] = y;
            feat[(size_t)b * FC_FS + k] = y;
        } else {
            fv[(size_t)b * PIX + k - 2 * PIX] = y;
            feat[(size_t)b * FC_FS + FC_KP + k - 2 * PIX] = y;
        }
    }
}

// fc data gradients with the feature ReLU masks (= the masked small_gemm dgrad) and the
// head BN-backward partial sums (= head_bn_bwd_partial_kernel), one workgroup per 32
// boards x 32 features (grid.y: 15 policy then 8 value feature tiles):
//   out[b][f] = S_k d[b][k] W[k][f],  d = dlogits (K = 225, W = policy_fc [225][450])
//                                     or dhv (K = 64, W = value_fc1 [64][225])
// The group's d rows are staged into LDS with coalesced loads (odd row stride: the
// MFMA's column reads spread over the banks); W is read straight into registers,
// W[k = 2s + h][f0 + lane] (128-B rows per half-wave), all of a wave's loads issued
// before the staging.  K split over the four waves, partial tiles summed in fixed wave
// order; per workgroup fp64 S dy, S (z - mean) dy of its head channel.
constexpr int HD_PT = (2 * PIX + 31) / 32;   // 15 policy feature tiles
constexpr int HD_VT = (PIX + 31) / 32;       // 8 value feature tiles
constexpr int HD_LDA = ACTIONS + 4;          // 229

__global__ __launch_bounds__(256) void head_dgrad_kernel(const HeadDgradArgs a)
{
    __shared__ float As[32][HD_LDA];
    __shared__ float red[4][16][64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    const int i0 = blockIdx.x * 32, ft = blockIdx.y;
    const bool val = ft >= HD_PT;
    const int f0 = val ? (ft - HD_PT) * 32 : ft * 32;
    const int F = val ? PIX : 2 * PIX;
    const int K = val ? VHID : ACTIONS;
    const float* W = val ? a.wv1 : a.wpf;
    const int f = f0 + r32;
    const bool fok = f < F;
    const int steps = (K + 1) / 2;
    const int s0 = wid * steps / 4, s1 = (wid + 1) * steps / 4;
    constexpr int SMAX = (ACTIONS + 1) / 2 / 4 + 1;   // 29
    float bw[SMAX];
#pragma unroll
    for (int u = 0; u < SMAX; ++u) {
        const int k = 2 * (s0 + u) + h;
        bw[u] = (s0 + u < s1 && k < K && fok) ? W[(size_t)k * F + f] : 0.f;
    }
    // every staging load of the thread in flight before its LDS stores
    auto stage = [&](const float* src, auto kc) {
        constexpr int KK = decltype(kc)::value, NE = (32 * KK + 255) / 256;
        float v[NE];
#pragma unroll
        for (int u = 0; u < NE; ++u) {
            const int e = tid + 256 * u, bb = e / KK;
            v[u] = (e < 32 * KK && i0 + bb < a.B) ? src[(size_t)i0 * KK + e] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < NE; ++u) {
            const int e = tid + 256 * u, bb = e / KK, k = e - bb * KK;
            if (e < 32 * KK) As[bb][k] = v[u];
        }
    };
    if (val) stage(a.dhv, std::integral_constant<int, VHID>{});
    else stage(a.dlogits, std::integral_constant<int, ACTIONS>{});
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int u = 0; u < SMAX; ++u)
        if (s0 + u < s1) {
            const int k = 2 * (s0 + u) + h;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(k < K ? As[r32][k] : 0.f, bw[u], acc, 0, 0, 0);
        }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wid][r][lane] = acc[r];
    __syncthreads();
    if (wid != 0) return;
    double hs[6] = {0, 0, 0, 0, 0, 0};   // (S dy, S (z - mean) dy) of head channels 0, 1, 2
    if (fok) {
        const int ch = val ? 2 : f < PIX ? 0 : 1;
        const double mu = (double)a.hmean[ch];
        double sd = 0.0, sq = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int b = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (b >= a.B) continue;
            const float v = ((red[0][r][lane] + red[1][r][lane]) + red[2][r][lane]) + red[3][r][lane];
            const float fe = val ? a.fv[(size_t)b * PIX + f] : a.fp[(size_t)b * 2 * PIX + f];
            const float zz = a.zh[(size_t)b * 3 * PIX + (val ? 2 * PIX : 0) + f];
            const float d = fe > 0.f ? v : 0.f;
            if (val) a.dfv[(size_t)b * PIX + f] = d;
            else a.dfp[(size_t)b * 2 * PIX + f] = d;
            sd += (double)d;
            sq += ((double)zz - mu) * (double)d;
        }
        hs[2 * ch] = sd;
        hs[2 * ch + 1] = sq;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) hs[k] = wsum_d(hs[k]);
    if (lane < 6) a.part[(size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 6 + lane] = hs[lane];
}

// head-BN backward finalize over head_dgrad_kernel's per-workgroup partials, one
// wave: lane g sums workgroups g, g + 64, ..., then a fixed xor tree; hk (optional):
// the [3][3] coefficients (S dy / N, k, invstd * gamma) for the caller's own use; write: publish dgamma / dbeta
__device__ __forceinline__ void head_bwd_fin_wave(const HeadDgradArgs& a, int nwg, float* hk, bool write)
{
    const int lane = threadIdx.x & 63;
    double sm[6] = {0, 0, 0, 0, 0, 0};
    for (int g = lane; g < nwg; g += 64)
#pragma unroll
        for (int k = 0; k < 6; ++k) sm[k] += a.part[(size_t)g * 6 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) sm[k] = wsum_d(sm[k]);
    if (lane < 3) {
        const int ch = lane;
        const BnDesc d = a.desc[ch < 2 ? a.pol_layer : a.val_layer];
        const int c = ch < 2 ? ch : 0;
        const double N = (double)a.B * PIX;
        const double sd = sm[2 * ch], qd = sm[2 * ch + 1];
        const float inv = a.hinv[ch];
        const double invd = (double)inv;
        const float k0 = (float)(sd / N), k1 = (float)(qd * invd * invd / N), k2 = inv * a.params[d.gamma_off + c];
        if (hk) {
            hk[ch * 3 + 0] = k0;
            hk[ch * 3 + 1] = k1;
            hk[ch * 3 + 2] = k2;
        }
        if (write) {
            a.grads[d.gamma_off + c] = (float)(qd * invd);
            a.grads[d.beta_off + c] = (float)sd;
            if (a.hb) {
                a.hb[ch * 3 + 0] = k0;
                a.hb[ch * 3 + 1] = k1;
                a.hb[ch * 3 + 2] = k2;
            }
        }
    }
}

// fc weight gradients dWpf[j][k] = S_b dlogits[b][j] fp[b][k] (225 x 450) and dWv1[u][k]
// = S_b dhv[b][u] fv[b][k] (64 x 225), K = the batch: one 32 x 32 output tile per
// workgroup (grid.x: 8 x 15 policy tiles, then 2 x 8 value tiles), K split over the
// four waves, both operands read straight into registers (A[j][b] = d[b][j] and
// B[b][k] = f[b][k]: 128-B row pieces per half-wave), partial tiles summed in fixed wave
// order through 16 KB of LDS -- small enough to share a CU with the conv weight-grad
// workgroups at the end of the step (small_gemm stages K in 131 KB and waits for a free CU)
constexpr int HW_PJ = (ACTIONS + 31) / 32, HW_PK = (2 * PIX + 31) / 32;   // 8 x 15 policy tiles
constexpr int HW_VJ = VHID / 32, HW_VK = (PIX + 31) / 32;                 // 2 x 8 value tiles

__global__ __launch_bounds__(256) void head_fc_wgrad_kernel(const float* __restrict__ dlogits,
                                                            const float* __restrict__ fp,
                                                            const float* __restrict__ dhv,
                                                            const float* __restrict__ fv, float* __restrict__ gpf,
                                                            float* __restrict__ gv1, int B)
{
    __shared__ float red[4][16][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    int t = blockIdx.x;
    const bool val = t >= HW_PJ * HW_PK;
    if (val) t -= HW_PJ * HW_PK;
    const int nk = val ? HW_VK : HW_PK;
    const int j0 = (t / nk) * 32, k0 = (t % nk) * 32;
    const int J = val ? VHID : ACTIONS, Kf = val ? PIX : 2 * PIX;
    const float* D = val ? dhv : dlogits;   // [B][J]
    const float* Fm = val ? fv : fp;        // [B][Kf]
    const int j = j0 + r32, k = k0 + r32;
    const bool jok = j < J, kok = k < Kf;
    const int steps = (B + 1) / 2;
    const int s0 = wid * steps / 4, s1 = (wid + 1) * steps / 4;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    constexpr int U = 16;   // steps per batch of loads
    for (int sb = s0; sb < s1; sb += U) {
        float av[U], bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int b = 2 * (sb + u) + h;
            const bool ok = sb + u < s1 && b < B;
            av[u] = ok && jok ? D[(size_t)b * J + j] : 0.f;
            bv[u] = ok && kok ? Fm[(size_t)b * Kf + k] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (sb + u < s1) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wid][r][lane] = acc[r];
    __syncthreads();
    if (wid == 0) {
        float* G = val ? gv1 : gpf;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = ((red[0][r][lane] + red[1][r][lane]) + red[2][r][lane]) + red[3][r][lane];
            const int jj = j0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (jj < J && kok) G[(size_t)jj * Kf + k] = v;
        }
    }
}

hipError_t launch_head_fc_wgrad(const float* dlogits, const float* fp, const float* dhv, const float* fv, float* gpf,
                                float* gv1, int B, hipStream_t st)
{
    hipLaunchKernelGGL(head_fc_wgrad_kernel, dim3(HW_PJ * HW_PK + HW_VJ * HW_VK), dim3(256), 0, st, dlogits, fp, dhv,
                       fv, gpf, gv1, B);
    return hipGetLastError();
}

int head_dgrad_groups(int B) { return ((B + 31) / 32) * (HD_PT + HD_VT); }

hipError_t launch_head_bn_apply_feat(float* fp, float* fv, float* feat, int B, const HeadStatsArgs& fin,
                                     hipStream_t st)
{
    // grid-stride: every workgroup reduces all M/64 statistics partials first, so the
    // grid is capped (256 workgroups: the reduction traffic stays linear in B)
    const int total = B * 3 * PIX;
    int nb = (total + 255) / 256;
    nb = nb > 256 ? 256 : nb;
    hipLaunchKernelGGL(head_bn_apply_feat_kernel, dim3(nb), dim3(256), 0, st, fin.zh, fp, fv, feat, B, fin,
                       head_proj_stats_groups(fin.M));
    return hipGetLastError();
}

// the projections + statistics partials (finalized by every workgroup of
// head_bn_apply_feat_kernel)
hipError_t launch_head_proj_partials(int C, bool apply, const HeadStatsArgs& a, hipStream_t st)
{
    const int nwg = head_proj_stats_groups(a.M);
#define AZG_HPQ(CC)                                                                                          \
    case CC:                                                                                                 \
        if (apply) hipLaunchKernelGGL((head_proj_stats_kernel<CC, true>), dim3(nwg), dim3(256), 0, st, a);  \
        else hipLaunchKernelGGL((head_proj_stats_kernel<CC, false>), dim3(nwg), dim3(256), 0, st, a);       \
        break;
    switch (C) {
        AZG_HPQ(64)
        AZG_HPQ(128)
        AZG_HPQ(256)
        default: return hipErrorInvalidValue;
    }
#undef AZG_HPQ
    return hipGetLastError();
}

__global__ __launch_bounds__(64) void head_bn_bwd_fin_kernel(const HeadDgradArgs a, int nwg)
{
    head_bwd_fin_wave(a, nwg, nullptr, true);
}

hipError_t launch_head_bwd_fin(const HeadDgradArgs& a, hipStream_t st)
{
    hipLaunchKernelGGL(head_bn_bwd_fin_kernel, dim3(1), dim3(64), 0, st, a, head_dgrad_groups(a.B));
    return hipGetLastError();
}

hipError_t launch_head_dgrad(const HeadDgradArgs& a, hipStream_t st)
{
    hipLaunchKernelGGL(head_dgrad_kernel, dim3((a.B + 31) / 32, HD_PT + HD_VT), dim3(256), 0, st, a);
    return hipGetLastError();
}

int head_proj_stats_groups(int M) { return (M + HP_ROWS - 1) / HP_ROWS; }

hipError_t launch_heads_bwd_fused(int C, bool bnx, const HeadBwdArgs& a, hipStream_t st)
{
    dim3 grid((a.M + 127) / 128);
#define AZG_HBF(CC)                                                                                     \
    case CC:                                                                                            \
        if (bnx) hipLaunchKernelGGL((heads_bwd_fused_kernel<CC, true>), grid, dim3(256), 0, st, a);    \
        else hipLaunchKernelGGL((heads_bwd_fused_kernel<CC, false>), grid, dim3(256), 0, st, a);       \
        return hipGetLastError();
    switch (C) {
        AZG_HBF(64)
        AZG_HBF(128)
        AZG_HBF(256)
        default: return hipErrorInvalidValue;
    }
#undef AZG_HBF
}

}  // namespace azg
