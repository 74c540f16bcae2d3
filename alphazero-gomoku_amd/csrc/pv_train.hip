// Train step of the policy/value net (reference network.py:199-235):
//   train-mode forward (BN batch statistics, running-stat update), log_softmax,
//   KLDivLoss(batchmean) + MSELoss, backward, clip_grad_norm_(3.0), Adam.
//
// Numerics follow ATen's CPU kernels the reference runs on:
//  * BN train stats: two-pass mean / biased var accumulated in double, invstd =
//    1/sqrt(var+eps) in double then stored fp32; y = x*alpha + beta with
//    alpha = invstd*gamma, beta = bias - mean*alpha; running stats updated in
//    double with the unbiased var (momentum 0.1).  Here: per-128-row tile (mean,
//    M2) in fp32, combined across tiles exactly in fp64.
//  * BN backward: sum = S dy, dotp = S (x-mean) dy, k = dotp*invstd^2/N,
//    dx = (dy - sum/N - (x-mean)*k) * invstd * gamma; dgamma = dotp*invstd.
//  * Adam (torch single-tensor path): g += wd*p; m.lerp_(g, 1-b1);
//    v = v*b2 + (1-b2)*g*g; denom = sqrt(v)/sqrt(bc2) + eps; p -= lr/bc1 * m/denom.
//  * clip_grad_norm_: total = ||grads||_2, coef = min(max_norm/(total+1e-6), 1),
//    grads *= coef (always).
//
// Schedule of one step (train_backward_t): stem (+ BN statistics from its accumulators)
// -> 12 x conv3x3_train (each applies the previous BN + ReLU (+ residual) in its halo
// staging and finalizes its own BN in its last workgroup) -> the head chain
// (pv_train_heads.hip) -> the tower backward on two streams (dgrads on the caller's,
// weight grads on a low-priority side stream) -> head weight grads, stem backward;
// train_apply: clip + Adam + the next step's weight packs.
#include "pv_internal.h"
#include "pv_halo.h"
#include "pv_train_heads.h"
#include "pv_wgrad.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

namespace azg {

hipError_t launch_wgrad(int C, const float* dz, const float* x, const int* rowtab, float* slab, float* dw, int M,
                        int S, hipStream_t st, bool reduce);
hipError_t launch_rowtab(int* rowtab, int n, hipStream_t st);
hipError_t launch_wgrad_reduce(int C, const float* slab, float* dw, int S, hipStream_t st);
int wgrad_splits(int C, int M);
constexpr int kMaxWgradSplits = 64;   // wgrad_splits <= slots / tiles <= 56, rounded to 8

constexpr int TROWS = 64;    // rows per tile of bn_bwd_reduce_kernel (a net without residual blocks)
constexpr int kApplyU = 4;   // float4 per thread and pass of the BN apply kernels
constexpr int HROWS = 128;   // rows per tile of the head-projection backward partials

int g_train_fuse_apply = 1;   // key 23: 1 BN applies folded into the next conv's staging; 0 separate passes
int g_train_fuse_fin = 1;     // key 24: 1 BN finalize by the last workgroup of the producing conv; 0 separate kernels
int g_train_apply_grid = 0;   // key 44: workgroup cap of the BN apply / BN-backward apply passes (0: one float4 per thread)

struct TrainWS {
    int cap = 0;
    std::vector<float*> allocs;
    float* z0 = nullptr;
    float* a0 = nullptr;
    std::vector<float*> z1, hh, z2, xo;
    float *gX = nullptr, *DH = nullptr, *GR = nullptr;
    std::vector<float*> dzs;     // one dZ buffer per backward conv (k = 2i + 1: conv2 of block i, 2i: conv1)
    float* wdpack = nullptr;     // dgrad-packed conv weights, 2*NB x 9*C*C
    float* wdpack16 = nullptr;   // the same split-fp16 (key 50), allocated on first use
    unsigned wd16_gen = ~0u;     // h3_gen it was packed from
    unsigned* dmax = nullptr;    // [2*NB] max |dz| bits of each dgrad input (zeroed per step)
    // per BN layer, at BnDesc::out_off (nfold floats each)
    float *bmean = nullptr, *binv = nullptr, *bscale = nullptr, *bshift = nullptr;
    float *bgm = nullptr, *bk = nullptr, *biw = nullptr;
    // partials
    float *part_a = nullptr, *part_b = nullptr;   // [ntile][C]
    float* hpart = nullptr;                        // [ntile][3][C]
    float* spart = nullptr;                        // [B][27][C]
    float* slab[2] = {nullptr, nullptr};           // weight-grad split-K slabs (two alternate)
    int slab_S = 0;                                // splits one slab holds
    int* rowtab = nullptr;                         // padded row of every pixel (weight grad v2)
    unsigned* fincnt = nullptr;   // fused BN finalize arrival counters, one per N tile
    // heads
    float *zh = nullptr, *fp = nullptr, *fv = nullptr, *hv = nullptr, *dpre = nullptr;
    float *dlogits = nullptr, *dfp = nullptr, *dfv = nullptr, *dhv = nullptr, *lossb = nullptr;
    double* hsp1 = nullptr;      // head_proj_stats_kernel partials [groups][6]
    double* hdp = nullptr;       // head_dgrad_kernel partials [groups][6]
    float* feat = nullptr;       // [B][FC_FS] head features, eval row layout (zero pads)
    float* pre = nullptr;        // [B][FC_OUT] fc pre-activations (logits | value hidden)
    float* hbw = nullptr;        // [3][3] head-BN backward coefficients (batches above kHeadFoldMaxB)
    // optimizer
    double* npart = nullptr;     // grad sq-sum partials
    float* scal = nullptr;       // [0] total norm, [1] clip coef
    // the BN running stats / num_batches_tracked the step in flight started from: a step
    // the Adam kernel skips (split-fp16 range overflow on some rank) restores them
    float* bn_bak = nullptr;
    int64_t* nbt_bak = nullptr;
    // two-stream backward: weight grads on `side`
    hipStream_t side = nullptr;
    hipEvent_t ev_ready = nullptr, ev_join = nullptr;
    // debug snapshots of gX (AZG_DEBUG_SNAP=1, two-stream schedule): after heads, after each block
    std::vector<float*> snap;
};

static TrainWS* ws_of(azg_pv* h) { return (TrainWS*)h->train; }

// the weight-grad stream of the two-stream schedule: lowest priority, so the dependent
// chain on the caller's stream is dispatched first whenever workgroup slots free up;
// its hand-off events release at device scope (they order two streams of one device)
static hipError_t make_side_stream(TrainWS* w)
{
    if (w->side && w->ev_ready && w->ev_join) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!w->side) {
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&w->side, hipStreamNonBlocking, least);
    }
    // each object is created only if missing: a failed creation is retried by the next
    // step instead of leaving a null event behind a live stream
    const unsigned flags = hipEventDisableTiming | hipEventReleaseToDevice;
    if (e == hipSuccess && !w->ev_ready) e = hipEventCreateWithFlags(&w->ev_ready, flags);
    if (e == hipSuccess && !w->ev_join) e = hipEventCreateWithFlags(&w->ev_join, flags);
    return e;
}

void free_train_workspace(azg_pv* h)
{
    TrainWS* w = ws_of(h);
    if (!w) return;
    if (w->side) (void)hipStreamSynchronize(w->side);
    for (float* p : w->allocs) (void)hipFree(p);
    if (w->ev_ready) (void)hipEventDestroy(w->ev_ready);
    if (w->ev_join) (void)hipEventDestroy(w->ev_join);
    if (w->side) (void)hipStreamDestroy(w->side);
    delete w;
    h->train = nullptr;
}

// ---------------------------------------------------------------------------
// kernels

__device__ __forceinline__ double block_sum_d(double v, double* red)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; ++i) s += red[i];
    __syncthreads();
    return s;
}

// a = relu(z*scale + shift [+ res]) over the interior of padded NHWC tensors
template <int C, bool RES, bool WT = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, const float* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ out,
                                                       int M)
{
    // grid-stride, kApplyU float4 per thread and pass, loads first (as bn_bwd_apply_kernel)
    constexpr int F4 = C / 4, U = kApplyU;
    const int total = M * F4;
    const int stride = gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, padded_bytes(M, C));
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = (i0 % F4) * 4;
    const f32x4 s = *(const f32x4*)(scale + c);
    const f32x4 t = *(const f32x4*)(shift + c);
    for (int ib = i0; ib < total; ib += U * stride) {
        f32x4 v[U], r[U];
        int o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = min(ib + u * stride, total - 1);
            o[u] = pad_off(i / F4, C) + c;
            v[u] = *(const f32x4*)(z + o[u]);
            if (RES) r[u] = *(const f32x4*)(res + o[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ib + u * stride >= total) break;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float y = fmaf(v[u][k], s[k], t[k]);   // same arithmetic as the conv staging prologue (ProX)
                if (RES) y += r[u][k];
                v[u][k] = fmaxf(y, 0.f);
            }
            store4<WT>(out, rs, o[u], v[u]);
        }
    }
}

// BN backward partial sums per tile: dy = g * (act > 0); S dy, S (z-mean) dy.
// Thread = 4 consecutive channels (f32x4) x RPT rows, fixed-order LDS reduction.
template <int C>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ g,
                                                            const float* __restrict__ act,
                                                            const float* __restrict__ z,
                                                            const float* __restrict__ mean, float* __restrict__ pa,
                                                            float* __restrict__ pb, int M)
{
    constexpr int Q = C / 4, RG = 256 / Q, RPT = TROWS / RG;
    __shared__ f32x4 red[2][RG][Q];
    const int q = threadIdx.x % Q, rg = threadIdx.x / Q;
    const int m0 = blockIdx.x * TROWS;
    const int rows = min(TROWS, M - m0);
    const f32x4 mu = *(const f32x4*)(mean + 4 * q);
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, d2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int r = rg + RG * i;
        if (r < rows) {
            const int o = pad_off(m0 + r, C) + 4 * q;
            const f32x4 gv = *(const f32x4*)(g + o);
            const f32x4 av = *(const f32x4*)(act + o);
            const f32x4 zv = *(const f32x4*)(z + o);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dy = av[k] > 0.f ? gv[k] : 0.f;
                s[k] += dy;
                d2[k] = fmaf(zv[k] - mu[k], dy, d2[k]);
            }
        }
    }
    red[0][rg][q] = s;
    red[1][rg][q] = d2;
    __syncthreads();
    if (rg == 0) {
        f32x4 a = red[0][0][q], b = red[1][0][q];
        for (int k = 1; k < RG; ++k) {
            a += red[0][k][q];
            b += red[1][k][q];
        }
        *(f32x4*)(pa + (size_t)blockIdx.x * C + 4 * q) = a;
        *(f32x4*)(pb + (size_t)blockIdx.x * C + 4 * q) = b;
    }
}

// Batch statistics / BN-backward sums of one BN layer from per-tile partials
// (pv_halo.h bn_fin_accum + bn_fin_combine8: wave w sums tile class w % 8 of 64
// channels in fp64, fixed combine order -- exactly what the last workgroup of a fused
// train conv runs, so both are bitwise identical).  64 channels per workgroup.
template <bool FWD>
__global__ __launch_bounds__(512) void bn_fin_tiles_kernel(const float* __restrict__ pa, const float* __restrict__ pb,
                                                          int ntile, int prow, int M, int C, int nch, FinX f)
{
    __shared__ double red[2 * 8 * 64];
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + ln;
    double v0 = 0.0, v1 = 0.0;
    if (c < nch) bn_fin_accum<FWD>(pa, pb, C, ntile, prow, M, c, wv, v0, v1);
    bn_fin_combine8<FWD>(v0, v1, red, M, c, c < nch, f);
}

// dz = ((dy - gm) - (z - mean)*k) * invstd*gamma ; optional gres = dy.
// dy = g * (act > 0).  MZ (a layer without a residual input: act = relu(fma(z, scale,
// shift)), the same expression as the forward's apply): the mask is formed from z and
// the layer's folded scale / shift instead of reading act -- bitwise the same mask,
// one 4-B-per-channel tensor less to read.
// (kApplyU = 4 float4 per thread measured fastest in the step: 2.843-2.851 ms vs 2.854-
// 2.861 at 2 and 2.864-2.871 at 1, scripts/gpu_r4m.sh)
template <int C, bool GRES, bool WT = false, bool MZ = false, int U = kApplyU>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ g, const float* __restrict__ act, const float* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ gm, const float* __restrict__ kk,
    const float* __restrict__ iw, float* __restrict__ dz, float* __restrict__ gres, int M,
    const float* __restrict__ fscale = nullptr, const float* __restrict__ fshift = nullptr,
    unsigned* __restrict__ dmax = nullptr)
{
    // grid-stride, kApplyU float4 per thread and pass with every load issued before the
    // first store; the stride is a multiple of C/4, so a thread's channels are fixed and
    // its per-channel coefficients are loaded once
    constexpr int F4 = C / 4;
    const int total = M * F4;
    const int stride = gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t rz = wt_rsrc(dz, padded_bytes(M, C));
    const __amdgpu_buffer_rsrc_t rg = wt_rsrc(GRES ? gres : dz, padded_bytes(M, C));
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = (i0 % F4) * 4;
    const f32x4 mu = *(const f32x4*)(mean + c);
    const f32x4 g_ = *(const f32x4*)(gm + c);
    const f32x4 k_ = *(const f32x4*)(kk + c);
    const f32x4 w_ = *(const f32x4*)(iw + c);
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sh = sc;
    if constexpr (MZ) {
        sc = *(const f32x4*)(fscale + c);
        sh = *(const f32x4*)(fshift + c);
    }
    float amax = 0.f;
    for (int ib = i0; ib < total; ib += U * stride) {
        f32x4 gv[U], zv[U], av[U];
        int o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = min(ib + u * stride, total - 1);
            o[u] = pad_off(i / F4, C) + c;
            gv[u] = *(const f32x4*)(g + o[u]);
            zv[u] = *(const f32x4*)(z + o[u]);
            if constexpr (!MZ) av[u] = *(const f32x4*)(act + o[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ib + u * stride >= total) break;
            if constexpr (MZ) {
#pragma unroll
                for (int q = 0; q < 4; ++q) av[u][q] = fmaf(zv[u][q], sc[q], sh[q]);
            }
            f32x4 out, dyv;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float dy;
                out[q] = bnbwd_elem(gv[u][q], av[u][q], zv[u][q], mu[q], g_[q], k_[q], w_[q], dy);
                dyv[q] = dy;
            }
            store4<WT>(dz, rz, o[u], out);
            if (GRES) store4<WT>(gres, rg, o[u], dyv);
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(out[0]), fabsf(out[1])), fmaxf(fabsf(out[2]), fabsf(out[3]))));
        }
    }
    // max |dz| of the layer (the split-fp16 dgrad's input scale, key 50): the bits of a
    // non-negative float order as the floats
    if (dmax) {
        amax = wave_max(amax);
        if ((threadIdx.x & 63) == 0) atomicMax(dmax, __float_as_uint(amax));
    }
}

// ---- heads, train mode (the chain itself: pv_train_heads.hip) ----

__device__ __forceinline__ double wave_sum_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// per board (one wave): log_softmax, KL term and dlogits; value head tail, (v-z)^2,
// dpre = 2(v-z)/B (1-v^2) and the masked value-hidden gradient.
__global__ __launch_bounds__(256) void heads_loss_kernel(
    const float* __restrict__ lpre, const float* __restrict__ bpf, const float* __restrict__ hpre,
    const float* __restrict__ bv1, const float* __restrict__ wv2, const float* __restrict__ bv2,
    const float* __restrict__ pis, const float* __restrict__ zs, float* __restrict__ dlogits,
    float* __restrict__ hv, float* __restrict__ dhv, float* __restrict__ dpre, float* __restrict__ lossb, int B,
    int lps = ACTIONS, int hps = VHID)
{
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    float lg[4];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        lg[t] = j < ACTIONS ? lpre[(size_t)b * lps + j] + bpf[j] : -INFINITY;
        mx = fmaxf(mx, lg[t]);
    }
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (lane + 64 * t < ACTIONS) se += expf(lg[t] - mx);
    se = wave_sum(se);
    const float lse = logf(se);
    const float* tp = pis + (size_t)b * ACTIONS;
    float kl = 0.f, st = 0.f, tv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        tv[t] = j < ACTIONS ? tp[j] : 0.f;
        if (j < ACTIONS) {
            const float lp = (lg[t] - mx) - lse;
            if (tv[t] > 0.f) kl += tv[t] * (logf(tv[t]) - lp);
            st += tv[t];
        }
    }
    kl = wave_sum(kl);
    st = wave_sum(st);
    const float invB = 1.f / (float)B;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        if (j < ACTIONS) {
            const float lp = (lg[t] - mx) - lse;
            dlogits[(size_t)b * ACTIONS + j] = (expf(lp) * st - tv[t]) * invB;
        }
    }
    const float hid = fmaxf(hpre[(size_t)b * hps + lane] + bv1[lane], 0.f);
    const float pre = wave_sum(wv2[lane] * hid) + bv2[0];
    const float v = tanhf(pre);
    const float z = zs[b];
    const float dv = 2.f * (v - z) / (float)B;
    const float dp = dv * (1.f - v * v);
    hv[(size_t)b * VHID + lane] = hid;
    dhv[(size_t)b * VHID + lane] = hid > 0.f ? dp * wv2[lane] : 0.f;
    if (lane == 0) {
        lossb[b * 2 + 0] = kl;
        lossb[b * 2 + 1] = (v - z) * (v - z);
        dpre[b] = dp;
    }
}

// bias / value_fc2 gradients and the loss means: one wave per output (fixed order)
constexpr int HSG_OUT = ACTIONS + VHID + VHID + 2;
__global__ __launch_bounds__(256) void heads_small_grads_kernel(
    const float* __restrict__ dlogits, const float* __restrict__ dhv, const float* __restrict__ dpre,
    const float* __restrict__ hv, const float* __restrict__ lossb, int B, float* __restrict__ g_pfb,
    float* __restrict__ g_v1b, float* __restrict__ g_v2w, float* __restrict__ g_v2b, float* __restrict__ losses,
    unsigned* __restrict__ ovf, float* __restrict__ skip)
{
    const int lane = threadIdx.x & 63;
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= HSG_OUT) return;
    if (o == HSG_OUT - 1) {
        // every forward conv of this step ran before this kernel (same stream): the split-
        // fp16 range flag of the step moves into the gradient buffer's skip slot, so a DP
        // all-reduce of the gradient carries it to every rank (train_apply skips the step
        // where it is nonzero), and is cleared for the next step
        if (lane == 0 && skip) {
            const unsigned f = ovf ? __hip_atomic_load(ovf + kTrainFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            *skip = f ? 1.f : 0.f;
            if (f) __hip_atomic_store(ovf + kTrainFlag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        double pl = 0.0, vl = 0.0;
        for (int b = lane; b < B; b += 64) {
            pl += (double)lossb[2 * b];
            vl += (double)lossb[2 * b + 1];
        }
        pl = wave_sum_d(pl);
        vl = wave_sum_d(vl);
        if (lane == 0) {
            const float plf = (float)(pl / (double)B), vlf = (float)(vl / (double)B);
            losses[0] = plf;
            losses[1] = vlf;
            losses[2] = plf + vlf;
        }
        return;
    }
    float s = 0.f;
    if (o < ACTIONS) {
        for (int b = lane; b < B; b += 64) s += dlogits[(size_t)b * ACTIONS + o];
    } else if (o < ACTIONS + VHID) {
        const int u = o - ACTIONS;
        for (int b = lane; b < B; b += 64) s += dhv[(size_t)b * VHID + u];
    } else if (o < ACTIONS + 2 * VHID) {
        const int u = o - ACTIONS - VHID;
        for (int b = lane; b < B; b += 64) s = fmaf(dpre[b], hv[(size_t)b * VHID + u], s);
    } else {
        for (int b = lane; b < B; b += 64) s += dpre[b];
    }
    s = wave_sum(s);
    if (lane == 0) {
        if (o < ACTIONS) g_pfb[o] = s;
        else if (o < ACTIONS + VHID) g_v1b[o - ACTIONS] = s;
        else if (o < ACTIONS + 2 * VHID) g_v2w[o - ACTIONS - VHID] = s;
        else g_v2b[0] = s;
    }
}

// out[j] = S_t part[t][j]: 64 outputs x 4 interleaved t-groups per workgroup,
// groups combined in fixed order.  mode 0: j < split -> out0[j], else out1[j-split];
// mode 1 (stem partials [t][k][c], j = k*C + c): out0[c*27 + k].
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ part, int T, int n,
                                                              float* __restrict__ out0, float* __restrict__ out1,
                                                              int split, int mode, int C)
{
    // 16 outputs x 16 t-phases per workgroup: every thread sums ~T/16 partials with
    // 8 loads in flight, then the 16 phases are added in fixed order
    constexpr int NJ = 16, NG = 16, UNR = 8;
    __shared__ float red[NG][NJ];
    const int jl = threadIdx.x % NJ, g = threadIdx.x / NJ;
    const int j = blockIdx.x * NJ + jl;
    float s = 0.f;
    if (j < n) {
        for (int t0 = g; t0 < T; t0 += NG * UNR) {
            float v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int t = t0 + NG * u;
                v[u] = t < T ? part[(size_t)t * n + j] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) s += v[u];
        }
    }
    red[g][jl] = s;
    __syncthreads();
    if (g == 0 && j < n) {
        float v = red[0][jl];
#pragma unroll
        for (int k = 1; k < NG; ++k) v += red[k][jl];
        if (mode == 0) {
            if (j < split) out0[j] = v;
            else out1[j - split] = v;
        } else {
            const int k = j / C, c = j - k * C;
            out0[c * 27 + k] = v;
        }
    }
}

// stem weight gradient partials per board: part[b][k][c] = S_p dz[p][c] * xpatch[p][k]
constexpr int STEM_WG_CHUNKS = 3;   // pixel chunks per board (75 pixels each) of the stem weight grad

// Stem weight grad partials: one workgroup per (board, 75-pixel chunk); thread =
// channel x pixel phase, 4 pixels' dz loads in flight; the board's padded input
// planes in LDS.  spart[(b * STEM_WG_CHUNKS + chunk) * 27 + k][C].
template <int C>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                         float* __restrict__ spart)
{
    __shared__ float xs[3 * PADPIX];
    constexpr int PCH = PIX / STEM_WG_CHUNKS;
    const int b = blockIdx.x / STEM_WG_CHUNKS, chunk = blockIdx.x % STEM_WG_CHUNKS, tid = threadIdx.x;
    const float* xb = x + (size_t)b * 3 * PIX;
    for (int i = tid; i < 3 * PADPIX; i += 256) {
        const int ci = i / PADPIX, rem = i - ci * PADPIX;
        const int yy = rem / PADW, xx = rem - yy * PADW;
        float v = 0.f;
        if (yy >= 1 && yy <= BOARD && xx >= 1 && xx <= BOARD) v = xb[ci * PIX + (yy - 1) * BOARD + (xx - 1)];
        xs[i] = v;
    }
    __syncthreads();
    constexpr int TPC = C < 256 ? 256 / C : 1;
    constexpr int UNR = 4;
    __shared__ float red[27][256];
    const int c = tid % C, rg = tid / C;
    if (C <= 256) {
        float acc[27];
#pragma unroll
        for (int k = 0; k < 27; ++k) acc[k] = 0.f;
        for (int i0 = rg; i0 < PCH; i0 += TPC * UNR) {
            float d[UNR];
            int yx[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = min(i0 + TPC * u, PCH - 1);
                const int p = chunk * PCH + i;
                const int y = p / BOARD, xq = p - y * BOARD;
                yx[u] = y * PADW + xq;
                d[u] = i0 + TPC * u < PCH ? dz[(size_t)(b * PADPIX + (y + 1) * PADW + (xq + 1)) * C + c] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u)
#pragma unroll
                for (int ci = 0; ci < 3; ++ci)
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx)
                            acc[ci * 9 + ky * 3 + kx] =
                                fmaf(d[u], xs[ci * PADPIX + yx[u] + ky * PADW + kx], acc[ci * 9 + ky * 3 + kx]);
        }
#pragma unroll
        for (int k = 0; k < 27; ++k) red[k][tid] = acc[k];
        __syncthreads();
        if (rg == 0) {
            for (int k = 0; k < 27; ++k) {
                float s = 0.f;
                for (int g = 0; g < TPC; ++g) s += red[k][g * C + c];
                spart[((size_t)blockIdx.x * 27 + k) * C + c] = s;
            }
        }
    }
}

// ---- optimizer --------------------------------------------------------------

__global__ __launch_bounds__(256) void grad_sqsum_kernel(const float* __restrict__ g, int64_t n,
                                                         double* __restrict__ part)
{
    __shared__ double red[8];
    double s = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = (double)g[i];
        s += v * v;
    }
    s = block_sum_d(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Adam with the clip_grad_norm_ finalize in its prologue: every workgroup reduces the
// grad_sqsum partials itself (one fixed-order block reduction, the same in every workgroup, so all
// workgroups hold the same coefficient, bitwise) and workgroup 0 publishes the norm --
// one launch boundary less on the step's critical path.
// The step's skip word (g[n], after any DP all-reduce: nonzero iff some rank's split-fp16
// train forward met an activation beyond fp16's range) decides, uniformly in every
// workgroup, whether the step commits: a skipped step leaves params, grads and moments
// as they are and restores the BN running stats and counters the step started from
// (BnKeep, saved when the previous step committed); a committed step saves them.
struct BnKeep {
    float* bn;            // running stats [nbn]
    float* bn_bak;
    int nbn;
    int64_t* nbt;         // num_batches_tracked [nlayers] (may be null)
    int64_t* nbt_bak;
    int nlayers;
    unsigned* skips;      // host-mapped count of skipped steps (azg_pv_train_status)
};
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const double* __restrict__ part, int nb, float max_norm,
                                                   float* __restrict__ scal, float* __restrict__ total_norm,
                                                   float lr_bc1, float b1w, float b2, float one_m_b2, float bc2_sqrt,
                                                   float eps, float wd, BnKeep k)
{
    const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, gstride = (int64_t)gridDim.x * blockDim.x;
    if (g[n] != 0.f) {   // skip: undo the step's running-stat updates
        for (int64_t i = gtid; i < k.nbn; i += gstride) k.bn[i] = k.bn_bak[i];
        if (k.nbt)
            for (int64_t i = gtid; i < k.nlayers; i += gstride) k.nbt[i] = k.nbt_bak[i];
        if (gtid == 0 && k.skips) __hip_atomic_fetch_add(k.skips, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    for (int64_t i = gtid; i < k.nbn; i += gstride) k.bn_bak[i] = k.bn[i];
    if (k.nbt)
        for (int64_t i = gtid; i < k.nlayers; i += gstride) k.nbt_bak[i] = k.nbt[i];
    __shared__ double red[8];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
    s = block_sum_d(s, red);
    const float tn = (float)sqrt(s);
    float coef = max_norm / (tn + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        scal[0] = tn;
        scal[1] = coef;
        if (total_norm) total_norm[0] = tn;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float gi = g[i] * coef;
        g[i] = gi;
        const float pi = p[i];
        if (wd != 0.f) gi = gi + wd * pi;
        float mi = m[i];
        mi = mi + b1w * (gi - mi);                 // lerp, weight < 0.5 branch
        float vi = v[i] * b2;
        vi = vi + one_m_b2 * gi * gi;              // addcmul
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = pi + (-lr_bc1) * (mi / denom);      // addcdiv
        m[i] = mi;
        v[i] = vi;
    }
}

// ---------------------------------------------------------------------------
// orchestration

static int32_t alloc_into(TrainWS* w, float** p, size_t floats, hipStream_t st, bool zero)
{
    hipError_t e = hipMalloc(p, floats * sizeof(float));
    if (e != hipSuccess) return set_error("train workspace: hipMalloc", e);
    w->allocs.push_back(*p);
    if (zero) {
        e = hipMemsetAsync(*p, 0, floats * sizeof(float), st);
        if (e != hipSuccess) return set_error("train workspace: hipMemsetAsync", e);
    }
    return 0;
}

static int32_t ensure_train_ws(azg_pv* h, int B, hipStream_t st)
{
    TrainWS* w = ws_of(h);
    if (w && w->cap >= B) return 0;
    int cap = w ? w->cap : 0;
    if (w) free_train_workspace(h);
    cap = cap ? cap : 128;
    while (cap < B) cap *= 2;
    w = new TrainWS();
    h->train = w;
    h->train_packs = false;   // a fresh dgrad pack buffer
    w->cap = cap;
    const int C = h->C, NB = h->NB;
    const size_t act = (size_t)cap * PADPIX * C;
    const int M = cap * PIX;
    const int ntile = (M + TROWS - 1) / TROWS;
    int32_t r = 0;
#define A(ptr, n, z) if ((r = alloc_into(w, &(ptr), (n), st, (z)))) return r
    A(w->z0, act, true);
    A(w->a0, act, true);
    w->z1.assign(NB, nullptr); w->hh.assign(NB, nullptr); w->z2.assign(NB, nullptr); w->xo.assign(NB, nullptr);
    for (int i = 0; i < NB; ++i) {
        A(w->z1[i], act, true);
        A(w->hh[i], act, true);
        A(w->z2[i], act, true);
        A(w->xo[i], act, true);
    }
    A(w->gX, act, true);
    A(w->DH, act, true);
    A(w->GR, act, true);
    w->dzs.assign(2 * NB, nullptr);
    for (int k = 0; k < 2 * NB; ++k) A(w->dzs[k], act, true);
    A(w->wdpack, (size_t)(2 * NB > 0 ? 2 * NB : 1) * 9 * C * C, false);
    {
        float* dm = nullptr;
        A(dm, (size_t)(2 * NB > 0 ? 2 * NB : 1), false);
        w->dmax = (unsigned*)dm;
    }
    const size_t nf = h->nfold;
    A(w->bmean, nf, true); A(w->binv, nf, true); A(w->bscale, nf, true); A(w->bshift, nf, true);
    A(w->bgm, nf, true); A(w->bk, nf, true); A(w->biw, nf, true);
    A(w->part_a, (size_t)ntile * C, false);
    A(w->part_b, (size_t)ntile * C, false);
    A(w->hpart, (size_t)((M + HROWS - 1) / HROWS) * 3 * C, false);
    A(w->spart, (size_t)cap * STEM_WG_CHUNKS * 27 * C, false);
    // slabs for the automatic split count at this capacity (or the key-27 override)
    w->slab_S = std::max(wgrad_splits(C, M), std::min(g_wgrad_splits, kMaxWgradSplits));
    for (int k = 0; k < 2; ++k) A(w->slab[k], (size_t)w->slab_S * 9 * C * C, false);
    {
        float* rt = nullptr;
        A(rt, (size_t)M + kRowTabPad, false);
        w->rowtab = (int*)rt;
    }
    if (hipError_t e = launch_rowtab(w->rowtab, M, st)) return set_error("train workspace: row table", e);
    A(w->zh, (size_t)cap * 3 * PIX, false);
    A(w->fp, (size_t)cap * 2 * PIX, false);
    A(w->fv, (size_t)cap * PIX, false);
    A(w->hv, (size_t)cap * VHID, false);
    A(w->dpre, (size_t)cap, false);
    A(w->dlogits, (size_t)cap * ACTIONS, false);
    A(w->dfp, (size_t)cap * 2 * PIX, false);
    A(w->dfv, (size_t)cap * PIX, false);
    A(w->dhv, (size_t)cap * VHID, false);
    A(w->lossb, (size_t)cap * 2, false);
    float* t = nullptr;
    A(t, 2 * 1024, false);
    w->npart = (double*)t;
    A(w->scal, 4, true);
    A(w->bn_bak, (size_t)h->nbn, false);
    A(t, 2 * h->bn_desc.size() + 2, false);
    w->nbt_bak = (int64_t*)t;
    h->bn_bak_ok = false;
    A(t, 4 * (2 * kTowerMaxBlocks + 2), true);
    w->fincnt = (unsigned*)t;
    A(t, (size_t)head_proj_stats_groups(M) * 6 * 2, false);
    w->hsp1 = (double*)t;
    A(t, (size_t)head_dgrad_groups(cap) * 6 * 2, false);
    w->hdp = (double*)t;
    A(w->feat, (size_t)cap * FC_FS, true);
    A(w->pre, (size_t)cap * FC_OUT, false);
    A(w->hbw, 16, false);
    if (getenv("AZG_DEBUG_SNAP")) {
        w->snap.assign(NB + 1, nullptr);
        for (int i = 0; i <= NB; ++i) A(w->snap[i], act, true);
    }
#undef A
    return 0;
}

static inline int grid_for(int64_t total) { int64_t b = (total + 255) / 256; return (int)(b > 8192 ? 8192 : b); }

#define AZG_CK(expr, what)                               \
    do {                                                 \
        hipError_t _e = (expr);                          \
        if (_e == hipSuccess) _e = hipGetLastError();    \
        if (_e != hipSuccess) return set_error(what, _e); \
    } while (0)

template <int C>
static int32_t train_backward_t(azg_pv* h, const float* x, const float* pis, const float* zs, int B,
                                float* losses, hipStream_t st)
{
    TrainWS* w = ws_of(h);
    const int NB = h->NB;
    const int M = B * PIX;
    const float* P = h->params;
    float* G = h->grads;
    const BnDesc* bd = h->bn_desc.data();
    const BnDesc* bdd = (const BnDesc*)h->bn_desc_dev;
    const int gM = g_train_apply_grid > 0 ? std::min(grid_for((int64_t)M * C / 4 / kApplyU), g_train_apply_grid)
                                          : grid_for((int64_t)M * C / 4 / kApplyU);
    const int ntt = (M + TRAIN_BM - 1) / TRAIN_BM;   // M tiles of conv3x3_train (partials per tile)
    const size_t CC9 = (size_t)9 * C * C;
    // the conv3x3_train launch that produces a layer's partials also finalizes it (key
    // 24; the fused and the separate finalize are bitwise identical)
    const bool ffin = g_train_fuse_fin != 0;

    // finalize arguments of one BN layer (forward statistics / backward sums)
    auto fin_args = [&](int layer, bool fwd) -> FinX {
        const BnDesc& d = bd[layer];
        FinX f{};
        f.gamma = P + d.gamma_off;
        if (fwd) {
            f.beta = P + d.beta_off;
            f.rmean = h->bn + d.stat_off;
            f.rvar = h->bn + d.stat_off + d.c;
            f.mean_o = w->bmean + d.out_off;
            f.inv_o = w->binv + d.out_off;
            f.scale_o = w->bscale + d.out_off;
            f.shift_o = w->bshift + d.out_off;
        } else {
            f.inv_i = w->binv + d.out_off;
            f.ggamma = G + d.gamma_off;
            f.gbeta = G + d.beta_off;
            f.gm_o = w->bgm + d.out_off;
            f.k_o = w->bk + d.out_off;
            f.iw_o = w->biw + d.out_off;
        }
        return f;
    };
    auto fin_fwd = [&](int layer, int prow, int nt) -> int32_t {
        hipLaunchKernelGGL(bn_fin_tiles_kernel<true>, dim3((bd[layer].c + 63) / 64), dim3(512), 0, st, w->part_a,
                           w->part_b, nt, prow, M, C, bd[layer].c, fin_args(layer, true));
        AZG_CK(hipGetLastError(), "train: bn_finalize_tiles");
        return 0;
    };
    auto bwd_fin = [&](int layer, int nt) -> int32_t {
        hipLaunchKernelGGL(bn_fin_tiles_kernel<false>, dim3((bd[layer].c + 63) / 64), dim3(512), 0, st,
                           w->part_a, w->part_b, nt, 1, M, C, bd[layer].c, fin_args(layer, false));
        AZG_CK(hipGetLastError(), "train: bn_bwd_finalize_tiles");
        return 0;
    };
    auto apply = [&](const float* z, const float* res, int layer, float* out) -> int32_t {
        const int o = bd[layer].out_off;
        if (res)
            hipLaunchKernelGGL((bn_apply_kernel<C, true, true>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        else
            hipLaunchKernelGGL((bn_apply_kernel<C, false, true>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        AZG_CK(hipGetLastError(), "train: bn_apply");
        return 0;
    };
    // train-mode conv: forward (z + BN tile statistics) or dgrad (+ BN-backward tile
    // sums of the layer below: act / z / layer `xl`); partials land in part_a / part_b;
    // fin >= 0: the BN layer this launch's partials belong to, finalized in-kernel
    auto conv = [&](int epi, int xe, const float* in, const float* wp, const float* res, float* out,
                    const float* xact, const float* xz, int xl, int fin, const float* osc = nullptr,
                    const unsigned* dmx = nullptr) -> int32_t {
        int pr = prof_begin(h, AZG_PROF_TRAIN_CONV, st, B);
        const EpiX ex{xact, xz, xl >= 0 ? w->bmean + bd[xl].out_off : nullptr, w->part_a, w->part_b};
        FinX fx{};
        if (fin >= 0) {
            fx = fin_args(fin, xe == XE_STATS);
            fx.cnt = w->fincnt;
        }
        AZG_CK(launch_conv3x3_train(C, epi, xe, in, wp, res, out, M, ex, st, nullptr, fin >= 0 ? &fx : nullptr, osc,
                                    osc && !dmx ? h->train_ovf_dev : nullptr, dmx),
               "train: conv3x3");
        prof_end(h, pr, st);
        return 0;
    };
    // dz = BN backward of `layer` applied to g; act == nullptr: a residual-free layer,
    // its ReLU mask from z and the layer's folded scale / shift (bn_bwd_apply MZ)
    auto bwd_apply = [&](const float* g, const float* act, const float* z, int layer, float* dz,
                         float* gres, unsigned* dmx = nullptr) -> int32_t {
        const int o = bd[layer].out_off;
#define AZG_BWD_APPLY(GR, MZ)                                                                                 \
        hipLaunchKernelGGL((bn_bwd_apply_kernel<C, GR, true, MZ>), dim3(gM), dim3(256), 0, st, g, act, z,     \
                           w->bmean + o, w->bgm + o, w->bk + o, w->biw + o, dz, gres, M, w->bscale + o,         \
                           w->bshift + o, dmx)
        if (gres) AZG_BWD_APPLY(true, false);
        else if (!act) AZG_BWD_APPLY(false, true);
        else AZG_BWD_APPLY(false, false);
#undef AZG_BWD_APPLY
        AZG_CK(hipGetLastError(), "train: bn_bwd_apply");
        return 0;
    };
    auto snap = [&](int k) -> int32_t {
        if (!w->snap.empty())
            AZG_CK(hipMemcpyAsync(w->snap[k], w->gX, (size_t)B * PADPIX * C * sizeof(float), hipMemcpyDeviceToDevice, st),
                   "train: snapshot");
        return 0;
    };
    int32_t r;
#define R(x) if ((r = (x))) return r

    // forward conv weights: the split-fp16 packs (key 49; ensured by train_backward) with
    // their per-layer 2^-e output factor, or the fp32 packs
    const bool fh3 = g_train_h3 && h->wpack16 && !h->train_fp32_once;
    auto fwd_w = [&](int ci) -> const float* {
        return fh3 ? (const float*)h->wpack16 + (size_t)ci * CC9 : h->wpack + (size_t)ci * CC9;
    };
    auto fwd_s = [&](int ci) -> const float* { return fh3 ? h->h3inv + (size_t)ci * C : nullptr; };
    // dgrad conv weights (key 50): the split-fp16 dgrad packs with the same 2^-e factor, the
    // input's 2^k from its max |dz| (w->dmax, zeroed at the step's start), or the fp32 packs
    const bool dh3 = g_train_dgrad_h3 && w->wdpack16 && h->h3inv && !h->train_fp32_once;
    auto dg_w = [&](int ci) -> const float* {
        return dh3 ? w->wdpack16 + (size_t)ci * CC9 : w->wdpack + (size_t)ci * CC9;
    };
    auto dg_s = [&](int ci) -> const float* { return dh3 ? h->h3inv + (size_t)ci * C : nullptr; };
    if (dh3 && NB > 0)
        AZG_CK(hipMemsetAsync(w->dmax, 0, (size_t)2 * NB * sizeof(unsigned), st), "train: dgrad max words");

    // ---- forward (train-mode BN) ----
    {
        int pr0 = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
        AZG_CK(launch_stem_stats(C, x, h->wstem, w->z0, B, w->part_a, w->part_b, st), "train: stem + statistics");
        R(fin_fwd(h->bn_stem, 128, (M + 127) / 128));
        prof_end(h, pr0, st);
    }
    const float* X = w->a0;
    // the last block's bn2 + residual + ReLU, left to the head projection kernel
    struct LastApply { const float* z; const float* res; int layer; float* out; } lastp{nullptr, nullptr, 0, nullptr};
    bool last_apply = false;
    // the staging prologue fits the 128-VGPR tile body at C <= 128; at C = 256 (eight
    // channel groups unrolled) it spills 96 VGPRs and costs ~1 ms per 10x256 step
    // (measured), so the separate apply passes stay there
    if (g_train_fuse_apply && C <= 128) {
        // every BN apply but the last is done by the next conv's halo staging
        // (pv_halo.h ProX): `pend` = the activation still to be formed from its raw z
        struct Pend { const float* z; int layer; const float* res; float* out; };
        Pend pend{w->z0, h->bn_stem, nullptr, w->a0};
        auto fused_conv = [&](const Pend& p, int ci, float* out, int fin) -> int32_t {
            int pr = prof_begin(h, AZG_PROF_TRAIN_CONV, st, B);
            const int o = bd[p.layer].out_off;
            const EpiX ex{nullptr, nullptr, nullptr, w->part_a, w->part_b};
            const ProX px{p.res, w->bscale + o, w->bshift + o, p.out};
            FinX fx = fin_args(fin, true);
            fx.cnt = w->fincnt;
            AZG_CK(launch_conv3x3_train(C, EPI_RAW, XE_STATS, p.z, fwd_w(ci), nullptr, out, M, ex, st, &px,
                                        ffin ? &fx : nullptr, fwd_s(ci), fh3 ? h->train_ovf_dev : nullptr),
                   "train: conv3x3 (fused BN apply)");
            prof_end(h, pr, st);
            if (!ffin) return fin_fwd(fin, TRAIN_BM, ntt);
            return 0;
        };
        for (int i = 0; i < NB; ++i) {
            R(fused_conv(pend, 2 * i, w->z1[i], h->bn_blk[i].first));
            pend = Pend{w->z1[i], h->bn_blk[i].first, nullptr, w->hh[i]};
            R(fused_conv(pend, 2 * i + 1, w->z2[i], h->bn_blk[i].second));
            pend = Pend{w->z2[i], h->bn_blk[i].second, X, w->xo[i]};
            X = w->xo[i];
        }
        if (pend.res) {
            last_apply = true;
            lastp = {pend.z, pend.res, pend.layer, pend.out};
        } else {
            R(apply(pend.z, pend.res, pend.layer, pend.out));
        }
    } else {
        R(apply(w->z0, nullptr, h->bn_stem, w->a0));
        for (int i = 0; i < NB; ++i) {
            const int l1 = h->bn_blk[i].first, l2 = h->bn_blk[i].second;
            R(conv(EPI_RAW, XE_STATS, X, fwd_w(2 * i), nullptr, w->z1[i], nullptr, nullptr, -1, ffin ? l1 : -1,
                   fwd_s(2 * i)));
            if (!ffin) R(fin_fwd(l1, TRAIN_BM, ntt));
            R(apply(w->z1[i], nullptr, l1, w->hh[i]));
            R(conv(EPI_RAW, XE_STATS, w->hh[i], fwd_w(2 * i + 1), nullptr, w->z2[i], nullptr, nullptr, -1,
                   ffin ? l2 : -1, fwd_s(2 * i + 1)));
            if (!ffin) R(fin_fwd(l2, TRAIN_BM, ntt));
            R(apply(w->z2[i], X, l2, w->xo[i]));
            X = w->xo[i];
        }
    }

    // ---- heads forward + loss + backward to the tower output (pv_train_heads.hip) ----
    const int hntile = (M + HROWS - 1) / HROWS;
    const int ho = bd[h->bn_pol].out_off;   // policy ch0, ch1, value: contiguous
    const float* wpf = P + h->poff[h->t_pfc_w];
    const float* wv1 = P + h->poff[h->t_vfc1_w];
    {
        int pr = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
        HeadStatsArgs hs{};
        hs.z = last_apply ? lastp.z : X;
        if (last_apply) {
            const int o = bd[lastp.layer].out_off;
            hs.res = lastp.res;
            hs.scale = w->bscale + o;
            hs.shift = w->bshift + o;
            hs.aout = lastp.out;
        }
        hs.wpc = P + h->poff[h->t_pc_w];
        hs.wvc = P + h->poff[h->t_vc_w];
        hs.zh = w->zh;
        hs.part = w->hsp1;
        hs.M = M;
        hs.desc = bdd;
        hs.pol_layer = h->bn_pol;
        hs.val_layer = h->bn_val;
        hs.params = P;
        hs.stats = h->bn;
        hs.bmean = w->bmean;
        hs.binv = w->binv;
        hs.bscale = w->bscale;
        hs.bshift = w->bshift;
        hs.nbt = h->nbt;
        hs.nbn = (int)h->bn_desc.size();
        AZG_CK(launch_head_proj_partials(C, last_apply, hs, st), "train: head_proj_partials");
        AZG_CK(launch_head_bn_apply_feat(w->fp, w->fv, w->feat, B, hs, st), "train: head_bn_apply_feat");
        AZG_CK(launch_heads_fc(w->feat, h->wfc, w->pre, B, st), "train: heads_fc");
        hipLaunchKernelGGL(heads_loss_kernel, dim3((B + 3) / 4), dim3(256), 0, st, w->pre, P + h->poff[h->t_pfc_b],
                           w->pre + ACTIONS, P + h->poff[h->t_vfc1_b], P + h->poff[h->t_vfc2_w],
                           P + h->poff[h->t_vfc2_b], pis, zs, w->dlogits, w->hv, w->dhv, w->dpre, w->lossb, B,
                           FC_OUT, FC_OUT);
        AZG_CK(hipGetLastError(), "train: heads_loss");
        HeadDgradArgs hd{};
        hd.dlogits = w->dlogits;
        hd.dhv = w->dhv;
        hd.wpf = wpf;
        hd.wv1 = wv1;
        hd.fp = w->fp;
        hd.fv = w->fv;
        hd.zh = w->zh;
        hd.hmean = w->bmean + ho;
        hd.dfp = w->dfp;
        hd.dfv = w->dfv;
        hd.part = w->hdp;
        hd.B = B;
        hd.desc = bdd;
        hd.pol_layer = h->bn_pol;
        hd.val_layer = h->bn_val;
        hd.params = P;
        hd.grads = G;
        hd.hinv = w->binv + ho;
        AZG_CK(launch_head_dgrad(hd, st), "train: head_dgrad");
        const bool fold_hb = B <= kHeadFoldMaxB;
        if (!fold_hb) {   // one wave finalizes; heads_bwd_fused reads the coefficients
            hd.hb = w->hbw;
            AZG_CK(launch_head_bwd_fin(hd, st), "train: head_bwd_fin");
        }
        HeadBwdArgs hw{};
        hw.act = X;
        hw.zh = w->zh;
        hw.dfp = w->dfp;
        hw.dfv = w->dfv;
        hw.hmean = w->bmean + ho;
        hw.wpc = P + h->poff[h->t_pc_w];
        hw.wvc = P + h->poff[h->t_vc_w];
        hw.gx = w->gX;
        hw.hpart = w->hpart;
        if (NB > 0) {
            hw.z2 = w->z2[NB - 1];
            hw.mean2 = w->bmean + bd[h->bn_blk[NB - 1].second].out_off;
            hw.pa = w->part_a;
            hw.pb = w->part_b;
        }
        hw.M = M;
        hw.dg = hd;
        hw.dg_nwg = fold_hb ? head_dgrad_groups(B) : 0;
        AZG_CK(launch_heads_bwd_fused(C, NB > 0, hw, st), "train: heads_bwd_fused");
        prof_end(h, pr, st);
    }
    R(snap(0));

    // ---- tower backward ----
    // The BN-backward sums of every layer but the last block's bn2 come out of the
    // epilogue of the dgrad conv that produces its gradient (XE_BNBWD, per 128-row
    // tile); the last block's bn2 sums come from heads_bwd_fused (per 128-row tile).
    bool done_fin = false;   // the stem's BN backward is finalized (by the last dgrad)
    bool side_used = false;
    if (NB > 0) R(bwd_fin(h->bn_blk[NB - 1].second, hntile));
    if (NB > 0) {
        // ---- the two-stream schedule: dgrads on the caller's stream, the
        // weight grads on `side` (one event hand-off per conv), each slab reduction
        // deferred behind the next conv's weight-grad kernel ----
        AZG_CK(make_side_stream(w), "train: side stream");
        const int S = wgrad_splits(C, M);
        if (S > w->slab_S) return set_error("train: wgrad splits exceed the slab workspace (key 27 above the allocation)", hipErrorInvalidValue);
        struct PendRed { float* slab; float* dw; } pend{nullptr, nullptr};
        int slab_i = 0;
        auto wgrad = [&](const float* dz, const float* xin, int tensor) -> int32_t {
            AZG_CK(hipEventRecord(w->ev_ready, st), "train: event record");
            AZG_CK(hipStreamWaitEvent(w->side, w->ev_ready, 0), "train: stream wait");
            int pr = prof_begin(h, AZG_PROF_TRAIN_WGRAD, w->side);
            float* sl = w->slab[slab_i];
            AZG_CK(launch_wgrad(C, dz, xin, w->rowtab, sl, nullptr, M, S, w->side, false), "train: wgrad");
            if (pend.slab) AZG_CK(launch_wgrad_reduce(C, pend.slab, pend.dw, S, w->side), "train: wgrad reduce");
            pend = PendRed{sl, G + h->poff[tensor]};
            slab_i ^= 1;
            prof_end(h, pr, w->side);
            side_used = true;
            return 0;
        };
        bool fin_next = true;   // the next layer's finalize is already done (the first: above)
        for (int i = NB - 1; i >= 0; --i) {
            const float* Xin = i == 0 ? w->a0 : w->xo[i - 1];
            const float* zin = i == 0 ? w->z0 : w->z2[i - 1];
            const int lin = i == 0 ? h->bn_stem : h->bn_blk[i - 1].second;
            const int l1 = h->bn_blk[i].first, l2 = h->bn_blk[i].second;
            float* dz2 = w->dzs[2 * i + 1];
            float* dz1 = w->dzs[2 * i];
            if (!fin_next) R(bwd_fin(l2, ntt));
            R(bwd_apply(w->gX, w->xo[i], w->z2[i], l2, dz2, w->GR, dh3 ? w->dmax + 2 * i + 1 : nullptr));
            R(wgrad(dz2, w->hh[i], h->t_blk[i].w2));
            R(conv(EPI_RAW, XE_BNBWD, dz2, dg_w(2 * i + 1), nullptr, w->DH, w->hh[i], w->z1[i], l1, ffin ? l1 : -1,
                   dg_s(2 * i + 1), dh3 ? w->dmax + 2 * i + 1 : nullptr));
            if (!ffin) R(bwd_fin(l1, ntt));
            R(bwd_apply(w->DH, nullptr, w->z1[i], l1, dz1, nullptr, dh3 ? w->dmax + 2 * i : nullptr));
            R(wgrad(dz1, Xin, h->t_blk[i].w1));
            R(conv(EPI_ADD, XE_BNBWD, dz1, dg_w(2 * i), w->GR, w->gX, Xin, zin, lin, ffin ? lin : -1, dg_s(2 * i),
                   dh3 ? w->dmax + 2 * i : nullptr));
            fin_next = ffin;
            R(snap(NB - i));
        }
        if (pend.slab) AZG_CK(launch_wgrad_reduce(C, pend.slab, pend.dw, S, w->side), "train: wgrad reduce");
        done_fin = ffin;
    }
    // ---- head weight grads (Adam's inputs only) ----
    AZG_CK(launch_head_fc_wgrad(w->dlogits, w->fp, w->dhv, w->fv, G + h->poff[h->t_pfc_w], G + h->poff[h->t_vfc1_w],
                                B, st),
           "train: head fc wgrad");
    hipLaunchKernelGGL(heads_small_grads_kernel, dim3((HSG_OUT + 3) / 4), dim3(256), 0, st, w->dlogits, w->dhv,
                       w->dpre, w->hv, w->lossb, B, G + h->poff[h->t_pfc_b], G + h->poff[h->t_vfc1_b],
                       G + h->poff[h->t_vfc2_w], G + h->poff[h->t_vfc2_b], losses, h->train_ovf_dev,
                       G + h->nparams);
    AZG_CK(hipGetLastError(), "train: heads_small_grads");
    // policy_conv.weight [2][C] then value_conv.weight [C]: partial layout [t][3][C]
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((3 * C + 15) / 16), dim3(256), 0, st, w->hpart, hntile, 3 * C,
                       G + h->poff[h->t_pc_w], G + h->poff[h->t_vc_w], 2 * C, 0, C);
    AZG_CK(hipGetLastError(), "train: heads proj wgrad");

    // ---- stem backward ----
    if (NB == 0) {
        const int ntile = (M + TROWS - 1) / TROWS;
        hipLaunchKernelGGL((bn_bwd_reduce_kernel<C>), dim3(ntile), dim3(256), 0, st, w->gX, w->a0, w->z0,
                           w->bmean + bd[h->bn_stem].out_off, w->part_a, w->part_b, M);
        AZG_CK(hipGetLastError(), "train: bn_bwd_reduce");
        R(bwd_fin(h->bn_stem, ntile));
    } else if (!done_fin) {
        R(bwd_fin(h->bn_stem, ntt));
    }
    R(bwd_apply(w->gX, nullptr, w->z0, h->bn_stem, w->DH, nullptr));
    hipLaunchKernelGGL((stem_wgrad_kernel<C>), dim3(B * STEM_WG_CHUNKS), dim3(256), 0, st, x, w->DH, w->spart);
    AZG_CK(hipGetLastError(), "train: stem_wgrad");
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((27 * C + 15) / 16), dim3(256), 0, st, w->spart, B * STEM_WG_CHUNKS, 27 * C,
                       G + h->poff[h->t_stem_w], nullptr, 27 * C, 1, C);
    AZG_CK(hipGetLastError(), "train: stem_wgrad_reduce");
    if (side_used) {   // the two-stream schedule: join the weight-grad stream
        AZG_CK(hipEventRecord(w->ev_join, w->side), "train: event record");
        AZG_CK(hipStreamWaitEvent(st, w->ev_join, 0), "train: stream wait");
    }
#undef R
    return 0;
}

int32_t train_backward(azg_pv* h, const float* x, const float* pis, const float* zs, int B, float* losses,
                       hipStream_t st)
{
    // a split-count override (key 27) above what the slabs were sized for: re-allocate
    if (TrainWS* w0 = ws_of(h); w0 && wgrad_splits(h->C, B * PIX) > w0->slab_S) free_train_workspace(h);
    if (int32_t r = ensure_train_ws(h, B, st)) return r;
    TrainWS* w = ws_of(h);
    // the packs are refreshed right after every Adam step (train_apply); a parameter
    // write the library did not see clears the flag (azg_pv_mark_dirty / bind)
    if (!h->train_packs) {
        if (int32_t r = repack(h, st, w->wdpack)) return r;
        h->train_packs = true;
    }
    if ((g_train_h3 || g_train_dgrad_h3) && !h->train_fp32_once)
        if (int32_t r = ensure_h3(h, st)) return r;
    // the split-fp16 dgrad packs follow every split-fp16 re-pack (same per-layer 2^e)
    if (g_train_dgrad_h3 && !h->train_fp32_once && h->NB > 0 && h->wpack16) {
        if (!w->wdpack16) {
            AZG_CK(hipMalloc(&w->wdpack16, (size_t)2 * h->NB * 9 * h->C * h->C * sizeof(float)),
                   "train: split-fp16 dgrad packs");
            w->allocs.push_back(w->wdpack16);
        }
        if (w->wd16_gen != h->h3_gen) {
            AZG_CK(launch_pack_h3_dgrad(h->params, h->conv_off_dev, 2 * h->NB, h->C, h->h3exp, w->wdpack16, st),
                   "train: split-fp16 dgrad pack");
            w->wd16_gen = h->h3_gen;
        }
    }
    // the running stats this step starts from (a skipped step restores them): refreshed
    // whenever they may have changed outside the library; a step the Adam kernel commits
    // refreshes them itself
    if (!h->bn_bak_ok) {
        AZG_CK(hipMemcpyAsync(w->bn_bak, h->bn, (size_t)h->nbn * sizeof(float), hipMemcpyDeviceToDevice, st),
               "train: BN backup");
        if (h->nbt)
            AZG_CK(hipMemcpyAsync(w->nbt_bak, h->nbt, h->bn_desc.size() * sizeof(int64_t), hipMemcpyDeviceToDevice, st),
                   "train: BN counter backup");
        h->bn_bak_ok = true;
    }
    const int C = h->C;
    int32_t r;
    switch (C) {
        case 64: r = train_backward_t<64>(h, x, pis, zs, B, losses, st); break;
        case 128: r = train_backward_t<128>(h, x, pis, zs, B, losses, st); break;
        case 256: r = train_backward_t<256>(h, x, pis, zs, B, losses, st); break;
        default: r = set_error("train: bad channels", hipErrorInvalidValue); break;
    }
    h->train_fp32_once = false;
    h->dirty = true;   // running stats changed -> eval fold must be redone
    return r;
}

int32_t train_apply(azg_pv* h, float* exp_avg, float* exp_avg_sq, int64_t step, float lr, float beta1, float beta2,
                    float eps, float wd, float max_norm, float* total_norm, hipStream_t st)
{
    if (int32_t r = ensure_train_ws(h, 1, st)) return r;
    TrainWS* w = ws_of(h);
    const int64_t n = h->nparams;
    const int nb = 1024;
    int pr = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
    hipLaunchKernelGGL(grad_sqsum_kernel, dim3(nb), dim3(256), 0, st, h->grads, n, w->npart);
    AZG_CK(hipGetLastError(), "apply: grad_sqsum");
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    const float lr_bc1 = (float)((double)lr / bc1);
    const float bc2_sqrt = (float)std::sqrt(bc2);
    // 1024 workgroups, grid-stride: each reduces the 1024 norm partials (8 KB) itself
    const BnKeep keep{h->bn, w->bn_bak, (int)h->nbn, h->nbt, w->nbt_bak, (int)h->bn_desc.size(),
                      h->train_ovf_dev ? h->train_ovf_dev + kTrainSkips : nullptr};
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n) < 1024 ? grid_for(n) : 1024), dim3(256), 0, st, h->params,
                       h->grads, exp_avg, exp_avg_sq, n, w->npart, nb, max_norm, w->scal, total_norm, lr_bc1,
                       (float)(1.0 - (double)beta1), beta2, (float)(1.0 - (double)beta2), bc2_sqrt, eps, wd, keep);
    AZG_CK(hipGetLastError(), "apply: adam");
    // every pack of the next step (and the eval BN fold) from the new parameters, on
    // this stream right behind Adam: the next train step starts without a repack
    h->train_packs = false;
    if (int32_t r = repack(h, st, w->wdpack)) return r;
    h->train_packs = true;
    h->dirty = false;
    prof_end(h, pr, st);
    return 0;
}

}  // namespace azg

namespace azg {
__global__ void unpad_kernel(const float* __restrict__ src, float* __restrict__ dst, int M, int C)
{
    const int total = M * C;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int m = i / C, c = i - m * C;
        dst[i] = src[pad_off(m, C) + c];
    }
}
}  // namespace azg

extern "C" int32_t azg_pv_debug_copy(azg_pv* h, int32_t which, int32_t index, float* dst, int32_t batch,
                                     void* stream)
{
    using namespace azg;
    TrainWS* w = ws_of(h);
    if (!w || batch > w->cap || !dst) return set_error("azg_pv_debug_copy: no train workspace / bad batch", hipSuccess);
    const float* src = nullptr;
    const bool blk = which >= 2 && which <= 5;
    if (blk && (index < 0 || index >= h->NB)) return set_error("azg_pv_debug_copy: bad block index", hipSuccess);
    switch (which) {
        case 0: src = w->z0; break;
        case 1: src = w->a0; break;
        case 2: src = w->z1[index]; break;
        case 3: src = w->hh[index]; break;
        case 4: src = w->z2[index]; break;
        case 5: src = w->xo[index]; break;
        case 6: src = w->gX; break;
        case 7:   // the last backward conv's dZ
            if (w->dzs.empty()) return set_error("azg_pv_debug_copy: no dZ (no residual blocks)", hipSuccess);
            src = w->dzs[0];
            break;
        case 8: src = w->DH; break;
        case 9: src = w->GR; break;
        case 10:
            if (index < 0 || index >= (int)w->snap.size()) return set_error("azg_pv_debug_copy: no snapshot (AZG_DEBUG_SNAP)", hipSuccess);
            src = w->snap[index];
            break;
        case 11: case 12: case 13: {   // head features, raw: fp [B][450], fv [B][225], hv [B][64]
            const float* hs = which == 11 ? w->fp : which == 12 ? w->fv : w->hv;
            const size_t n = (size_t)batch * (which == 11 ? 2 * PIX : which == 12 ? PIX : VHID);
            hipError_t e = hipMemcpyAsync(dst, hs, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream);
            return e == hipSuccess ? 0 : set_error("azg_pv_debug_copy", e);
        }
        default: return set_error("azg_pv_debug_copy: bad buffer id", hipSuccess);
    }
    const int M = batch * PIX;
    hipLaunchKernelGGL(unpad_kernel, dim3(grid_for((int64_t)M * h->C)), dim3(256), 0, (hipStream_t)stream, src, dst,
                       M, h->C);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error("azg_pv_debug_copy", e);
}

extern "C" int32_t azg_pv_train_backward(azg_pv* h, const float* x, const float* pis, const float* zs,
                                         int32_t batch, float* losses, void* stream)
{
    if (!h || !h->params || !h->grads) return azg::set_error("azg_pv_train_backward: handle not bound with grads", hipSuccess);
    if (!x || !pis || !zs || !losses) return azg::set_error("azg_pv_train_backward: null argument", hipSuccess);
    if (batch < 2) return azg::set_error("azg_pv_train_backward: batch must be >= 2 (train-mode BatchNorm)", hipSuccess);
    return azg::train_backward(h, x, pis, zs, batch, losses, (hipStream_t)stream);
}

extern "C" int32_t azg_pv_train_apply(azg_pv* h, float* exp_avg, float* exp_avg_sq, int64_t step, float lr,
                                      float beta1, float beta2, float eps, float weight_decay, float max_norm,
                                      float* total_norm, void* stream)
{
    if (!h || !h->params || !h->grads) return azg::set_error("azg_pv_train_apply: handle not bound with grads", hipSuccess);
    if (!exp_avg || !exp_avg_sq) return azg::set_error("azg_pv_train_apply: null moments", hipSuccess);
    if (step < 1) return azg::set_error("azg_pv_train_apply: step must be >= 1", hipSuccess);
    return azg::train_apply(h, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, weight_decay, max_norm, total_norm,
                            (hipStream_t)stream);
}

