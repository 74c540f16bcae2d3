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
#include "pv_internal.h"
#include "pv_halo.h"
#include "pv_train_heads.h"

#include <cmath>
#include <cstdlib>
#include <vector>

namespace azg {

hipError_t launch_wgrad(int C, const float* dz, const float* x, float* slab, float* dw, int M, int S,
                        hipStream_t st, bool reduce = true, unsigned* gcnt = nullptr, float* gslab = nullptr);
bool wgrad_comb_on(int kernel, int S);
hipError_t launch_wgrad_reduce(int C, const float* slab, float* dw, int S, hipStream_t st);
hipError_t launch_wgrad_reduce2(int C, const float* slab0, float* dw0, int S0, const float* slab1, float* dw1,
                                int S1, hipStream_t st);
int wgrad_splits(int C, int M);
constexpr int kMaxWgradSplits = 64;   // wgrad_splits <= slots / tiles <= 56, rounded to 8

constexpr int TROWS = 64;    // rows per statistics tile (BN stats / BN backward partials)
constexpr int HROWS = 128;   // rows per tile of the head-projection backward partials

struct TrainWS {
    int cap = 0;
    std::vector<float*> allocs;
    float* z0 = nullptr;
    float* a0 = nullptr;
    std::vector<float*> z1, hh, z2, xo;
    float *gX = nullptr, *DZ = nullptr, *DH = nullptr, *GR = nullptr;
    float* wdpack = nullptr;     // dgrad-packed conv weights, 2*NB x 9*C*C
    // per BN layer, at BnDesc::out_off (nfold floats each)
    float *bmean = nullptr, *binv = nullptr, *bscale = nullptr, *bshift = nullptr;
    float *bgm = nullptr, *bk = nullptr, *biw = nullptr;
    // partials
    float *part_a = nullptr, *part_b = nullptr;   // [ntile][C]
    float* hpart = nullptr;                        // [ntile][3][C]
    float* spart = nullptr;                        // [B][27][C]
    float* slab = nullptr;                         // wgrad split-K slabs
    float* slab2 = nullptr;                        // the second slab buffer (deferred reductions, key 39)
    float* gslab[2] = {nullptr, nullptr};          // split-group slabs [8][9][C][C] (key 41), alternating
    unsigned* gcnt = nullptr;                      // split-group arrival counters (key 41)
    int S = 0, rps = 0;
    unsigned* fincnt = nullptr;                    // fused BN finalize: arrival counters per N tile
    // heads
    float *zh = nullptr, *fp = nullptr, *fv = nullptr, *hv = nullptr, *dpre = nullptr;
    float *dlogits = nullptr, *dfp = nullptr, *dfv = nullptr, *dhv = nullptr, *dzh = nullptr, *lossb = nullptr;
    float *lpre = nullptr, *hpre = nullptr, *hbw = nullptr;   // FC pre-activations, head BN bwd coefficients
    double* hspart = nullptr;                                 // head BN (channel, chunk) partials
    // fused head chain (pv_train_heads.hip): per-workgroup partials + arrival counters
    double* hsp1 = nullptr;      // head_proj_stats_kernel [groups][6]
    double* hpd = nullptr;       // head_board_kernel [groups][head_board_pd()]
    float* hpf = nullptr;        // head_board_kernel [groups][head_board_pf()]
    unsigned* hcnt = nullptr;    // [3] arrival counters (0 between launches)
    double* hdp = nullptr;       // head_dgrad_kernel [groups][6]
    float* feat = nullptr;       // [B][FC_FS] head features, eval row layout (zero pads)
    float* pre = nullptr;        // [B][FC_OUT] fc pre-activations (logits | value hidden)
    // optimizer
    double* npart = nullptr;     // grad sq-sum partials
    float* scal = nullptr;       // [0] total norm, [1] clip coef
    // debug snapshots of gX (AZG_DEBUG_SNAP=1): after heads, after each block
    std::vector<float*> snap;
    // tower backward: the weight gradient of each conv runs on `side`, concurrently
    // with the data gradient on the caller's stream (both only read dZ); dZ
    // alternates between DZ and DZ2 so the next BN backward never overwrites a dZ a
    // pending wgrad still reads (ev_ready: dZ written; ev_done: its wgrad finished)
    float* DZ2 = nullptr;
    // key 34: one dZ buffer per conv (no reuse waits on the caller's stream: every
    // stream wait is a ~6 us bubble there, measured)
    std::vector<float*> dzs;
    hipStream_t side = nullptr;
    hipEvent_t ev_ready[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
    // split repack at the start of a step: the stem on the caller's stream, the rest on
    // `side` (ev_pack_in: the step's inputs are ready; ev_pack: the packs are written)
    hipEvent_t ev_pack_in = nullptr, ev_pack = nullptr;
    bool pack_pending = false;
    // the join of everything `side` ran before the optimizer (ev_join)
    hipEvent_t ev_join = nullptr;
    int ev_flags = -1;           // flags the hand-off events were created with (key 33)
    int side_prio = -1;          // priority class `side` was created with (key 37)
};

int g_train_dz_all = 1;     // key 34: 1 one dZ buffer per conv (default); 0 two alternating buffers + reuse waits
int g_train_pack_after = 1; // key 36: 1 the next step's weight packs right after Adam (same stream, no hand-off); 0 at the step start
int g_train_late_store = 1;    // key 42: 1 forward conv tiles stored after the BN-partial arrival count; 0 before
int g_train_fuse_bwd = 0;      // key 40: 1 conv1's BN backward in its dgrad staging (C <= 128); 0 bn_bwd_apply pass
int g_train_defer_reduce = 1;  // key 39: 1 each weight grad's slab reduction after the next conv's weight-grad kernel;
                               // 2 the same, the last two convs' reductions in one launch on the caller's stream after
                               // the join (+0.4 %, measured); 0 each right behind its own weight grad
int g_train_stem_stats = 1;  // key 38: 1 stem BN statistics from the stem's accumulators (default); 0 col_stats pass
int g_train_side_prio = 0;   // key 37: priority of the weight-grad stream: 0 lowest (default), 1 highest
int g_train_ev_device = 1;   // key 33: 1 stream hand-off events release at device scope (default); 0 system scope

// (re)create the stream hand-off events: they only order work between two streams of
// one device, so a device-scope release is enough (hipEventReleaseToDevice); the
// default system-scope release adds an L2 writeback + invalidate per record
static hipError_t make_side_stream(TrainWS* w)
{
    if (w->side && w->side_prio == g_train_side_prio) return hipSuccess;
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    if (w->side) {
        (void)hipStreamSynchronize(w->side);
        (void)hipStreamDestroy(w->side);
        w->side = nullptr;
    }
    e = hipStreamCreateWithPriority(&w->side, hipStreamNonBlocking, g_train_side_prio ? greatest : least);
    if (e == hipSuccess) w->side_prio = g_train_side_prio;
    return e;
}

static hipError_t make_events(TrainWS* w)
{
    const int flags = hipEventDisableTiming | (g_train_ev_device ? hipEventReleaseToDevice : 0);
    if (w->ev_flags == flags) return hipSuccess;
    hipEvent_t* evs[] = {&w->ev_ready[0], &w->ev_ready[1], &w->ev_done[0], &w->ev_done[1], &w->ev_pack_in,
                         &w->ev_pack, &w->ev_join};
    if (w->side) (void)hipStreamSynchronize(w->side);
    for (hipEvent_t* e : evs) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    for (hipEvent_t* e : evs) {
        hipError_t r = hipEventCreateWithFlags(e, flags);
        if (r != hipSuccess) return r;
    }
    w->ev_flags = flags;
    return hipSuccess;
}

static TrainWS* ws_of(azg_pv* h) { return (TrainWS*)h->train; }

void free_train_workspace(azg_pv* h)
{
    TrainWS* w = ws_of(h);
    if (!w) return;
    if (w->side) (void)hipStreamSynchronize(w->side);
    for (float* p : w->allocs) (void)hipFree(p);
    for (int i = 0; i < 2; ++i) {
        if (w->ev_ready[i]) (void)hipEventDestroy(w->ev_ready[i]);
        if (w->ev_done[i]) (void)hipEventDestroy(w->ev_done[i]);
    }
    if (w->ev_pack_in) (void)hipEventDestroy(w->ev_pack_in);
    if (w->ev_pack) (void)hipEventDestroy(w->ev_pack);
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

// per-tile column (mean, M2) of a padded NHWC tensor.  Thread = 4 consecutive
// channels (f32x4) x RPT rows held in registers: one HBM read, two passes from
// registers (exact two-pass M2 per tile), fixed-order LDS reduction.
template <int C>
__global__ __launch_bounds__(256) void col_stats_kernel(const float* __restrict__ z, float* __restrict__ pmean,
                                                        float* __restrict__ pm2, int M)
{
    constexpr int Q = C / 4, RG = 256 / Q, RPT = TROWS / RG;
    __shared__ f32x4 red[RG][Q];
    const int q = threadIdx.x % Q, rg = threadIdx.x / Q;
    const int m0 = blockIdx.x * TROWS;
    const int rows = min(TROWS, M - m0);
    f32x4 v[RPT];
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int r = rg + RG * i;
        v[i] = r < rows ? *(const f32x4*)(z + pad_off(m0 + r, C) + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        s += v[i];
    }
    red[rg][q] = s;
    __syncthreads();
    f32x4 tot = red[0][q];
    for (int g = 1; g < RG; ++g) tot += red[g][q];
    f32x4 mean;
#pragma unroll
    for (int k = 0; k < 4; ++k) mean[k] = tot[k] / (float)rows;
    __syncthreads();
    f32x4 m2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        if (rg + RG * i < rows) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = v[i][k] - mean[k];
                m2[k] = fmaf(d, d, m2[k]);
            }
        }
    }
    red[rg][q] = m2;
    __syncthreads();
    if (rg == 0) {
        f32x4 t = red[0][q];
        for (int g = 1; g < RG; ++g) t += red[g][q];
        *(f32x4*)(pmean + (size_t)blockIdx.x * C + 4 * q) = mean;
        *(f32x4*)(pm2 + (size_t)blockIdx.x * C + 4 * q) = t;
    }
}

// a = relu(z*scale + shift [+ res]) over the interior of padded NHWC tensors
template <int C, bool RES, bool WT = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, const float* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ out,
                                                       int M)
{
    constexpr int F4 = C / 4;
    const int total = M * F4;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, padded_bytes(M, C));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int m = i / F4, c = (i - m * F4) * 4;
        const int o = pad_off(m, C) + c;
        f32x4 v = *(const f32x4*)(z + o);
        const f32x4 s = *(const f32x4*)(scale + c);
        const f32x4 t = *(const f32x4*)(shift + c);
        f32x4 r;
        if (RES) r = *(const f32x4*)(res + o);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float y = fmaf(v[k], s[k], t[k]);   // same arithmetic as the conv staging prologue (ProX)
            if (RES) y += r[k];
            v[k] = fmaxf(y, 0.f);
        }
        store4<WT>(out, rs, o, v);
    }
}

// BN backward partial sums per tile: dy = g * (act > 0); S dy, S (z-mean) dy.
// Same thread layout as col_stats_kernel (f32x4 channels, fixed-order reduction).
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

// fixed-order fp64 block sum of NV values per thread (256 threads, 4 waves):
// wave shuffles, then the 4 wave sums in wave order
template <int NV>
__device__ __forceinline__ void block_sum4_d(double (&v)[NV], double (*red)[4])
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k][wid] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
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
template <int C, bool GRES, bool WT = false, bool MZ = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ g, const float* __restrict__ act, const float* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ gm, const float* __restrict__ kk,
    const float* __restrict__ iw, float* __restrict__ dz, float* __restrict__ gres, int M,
    const float* __restrict__ fscale = nullptr, const float* __restrict__ fshift = nullptr)
{
    constexpr int F4 = C / 4;
    const int total = M * F4;
    const __amdgpu_buffer_rsrc_t rz = wt_rsrc(dz, padded_bytes(M, C));
    const __amdgpu_buffer_rsrc_t rg = wt_rsrc(GRES ? gres : dz, padded_bytes(M, C));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int m = i / F4, c = (i - m * F4) * 4;
        const int o = pad_off(m, C) + c;
        const f32x4 gv = *(const f32x4*)(g + o);
        const f32x4 zv = *(const f32x4*)(z + o);
        f32x4 av;
        if constexpr (MZ) {
            const f32x4 sc = *(const f32x4*)(fscale + c), sh = *(const f32x4*)(fshift + c);
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = fmaf(zv[q], sc[q], sh[q]);
        } else {
            av = *(const f32x4*)(act + o);
        }
        const f32x4 mu = *(const f32x4*)(mean + c);
        const f32x4 g_ = *(const f32x4*)(gm + c);
        const f32x4 k_ = *(const f32x4*)(kk + c);
        const f32x4 w_ = *(const f32x4*)(iw + c);
        f32x4 out, dyv;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dy = av[q] > 0.f ? gv[q] : 0.f;
            dyv[q] = dy;
            out[q] = ((dy - g_[q]) - (zv[q] - mu[q]) * k_[q]) * w_[q];
        }
        store4<WT>(dz, rz, o, out);
        if (GRES) store4<WT>(gres, rg, o, dyv);
    }
}

// ---- heads (policy_conv/value_conv 1x1 -> BN -> ReLU -> FCs), train mode ----
constexpr int HSC = 32;   // chunks per head channel for the head BN reductions

__device__ __forceinline__ double wave_sum_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// per (channel, chunk): S z, S z^2 in double over the chunk of the B*225 pixels
__global__ __launch_bounds__(256) void head_stats_partial_kernel(const float* __restrict__ zh, int B,
                                                                 double* __restrict__ part)
{
    __shared__ double red[8];
    const int ch = blockIdx.x, chunk = blockIdx.y;
    const int N = B * PIX;
    const int i0 = (int)((int64_t)chunk * N / HSC), i1 = (int)((int64_t)(chunk + 1) * N / HSC);
    double s = 0.0, ss = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const int b = i / PIX, p = i - b * PIX;
        const double v = (double)zh[(b * 3 + ch) * PIX + p];
        s += v;
        ss += v * v;
    }
    s = block_sum_d(s, red);
    ss = block_sum_d(ss, red);
    if (threadIdx.x == 0) {
        part[(ch * HSC + chunk) * 2 + 0] = s;
        part[(ch * HSC + chunk) * 2 + 1] = ss;
    }
}

// batch stats of the 3 head BN channels -> folded coefficients + running stats
// Also advances every BN layer's num_batches_tracked (int64, bound with
// azg_pv_bind_counters) by one: the train-mode forward's counter update.
__global__ void head_stats_finalize_kernel(const double* __restrict__ part, int B, const BnDesc* desc, int pol_layer,
                                           int val_layer, const float* __restrict__ params,
                                           float* __restrict__ stats, float* __restrict__ bmean,
                                           float* __restrict__ binv, float* __restrict__ bscale,
                                           float* __restrict__ bshift, int64_t* __restrict__ nbt, int nbn)
{
    if (nbt)
        for (int i = threadIdx.x; i < nbn; i += blockDim.x) nbt[i] += 1;
    const int ch = threadIdx.x;
    if (ch >= 3) return;
    const BnDesc d = desc[ch < 2 ? pol_layer : val_layer];
    const int c = ch < 2 ? ch : 0;
    const double N = (double)B * PIX;
    double s = 0.0, ss = 0.0;
    for (int k = 0; k < HSC; ++k) {
        s += part[(ch * HSC + k) * 2 + 0];
        ss += part[(ch * HSC + k) * 2 + 1];
    }
    const double mean = s / N;
    double q = ss - s * mean;              // S (z - mean)^2
    q = q > 0.0 ? q : 0.0;
    const double var = q / N;
    const float mean_f = (float)mean;
    const float inv_f = (float)(1.0 / sqrt(var + (double)BN_EPS));
    const float alpha = inv_f * params[d.gamma_off + c];
    bmean[d.out_off + c] = mean_f;
    binv[d.out_off + c] = inv_f;
    bscale[d.out_off + c] = alpha;
    bshift[d.out_off + c] = params[d.beta_off + c] - mean_f * alpha;
    const double unb = N > 1 ? q / (N - 1.0) : var;
    float* rm = stats + d.stat_off;
    float* rv = stats + d.stat_off + d.c;
    rm[c] = (float)((double)BN_MOMENTUM * mean + (1.0 - (double)BN_MOMENTUM) * (double)rm[c]);
    rv[c] = (float)((double)BN_MOMENTUM * unb + (1.0 - (double)BN_MOMENTUM) * (double)rv[c]);
}

// fp[b][0..449] = relu(BN(zh policy)), fv[b][0..224] = relu(BN(zh value))
__global__ __launch_bounds__(256) void head_bn_apply_kernel(const float* __restrict__ zh,
                                                            const float* __restrict__ hscale,
                                                            const float* __restrict__ hshift, float* __restrict__ fp,
                                                            float* __restrict__ fv, int B)
{
    const int total = B * 3 * PIX;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int b = i / (3 * PIX), k = i - b * 3 * PIX;
        const int ch = k / PIX;
        const float y = fmaxf(zh[i] * hscale[ch] + hshift[ch], 0.f);
        if (ch < 2) fp[(size_t)b * 2 * PIX + k] = y;
        else fv[(size_t)b * PIX + k - 2 * PIX] = y;
    }
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
    float* __restrict__ g_v1b, float* __restrict__ g_v2w, float* __restrict__ g_v2b, float* __restrict__ losses)
{
    const int lane = threadIdx.x & 63;
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= HSG_OUT) return;
    if (o == HSG_OUT - 1) {
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

// head BN backward, (channel, chunk) partials: S dy, S (z-mean) dy in double
__global__ __launch_bounds__(256) void head_bn_bwd_partial_kernel(const float* __restrict__ zh,
                                                                  const float* __restrict__ dfp,
                                                                  const float* __restrict__ dfv, int B,
                                                                  const float* __restrict__ hmean,
                                                                  double* __restrict__ part)
{
    __shared__ double red[8];
    const int ch = blockIdx.x, chunk = blockIdx.y;
    const int N = B * PIX;
    const int i0 = (int)((int64_t)chunk * N / HSC), i1 = (int)((int64_t)(chunk + 1) * N / HSC);
    const double mu = (double)hmean[ch];
    double s = 0.0, q = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const int b = i / PIX, p = i - b * PIX;
        const double dy = ch < 2 ? (double)dfp[(size_t)b * 2 * PIX + ch * PIX + p] : (double)dfv[(size_t)b * PIX + p];
        s += dy;
        q += ((double)zh[(b * 3 + ch) * PIX + p] - mu) * dy;
    }
    s = block_sum_d(s, red);
    q = block_sum_d(q, red);
    if (threadIdx.x == 0) {
        part[(ch * HSC + chunk) * 2 + 0] = s;
        part[(ch * HSC + chunk) * 2 + 1] = q;
    }
}

// gamma/beta grads of the head BNs and the per-channel backward coefficients
// hb[ch][0..2] = (S dy / N, S(z-mean)dy invstd^2 / N, invstd*gamma)
__global__ void head_bn_bwd_finalize_kernel(const double* __restrict__ part, int B, const BnDesc* desc,
                                            int pol_layer, int val_layer, const float* __restrict__ params,
                                            float* __restrict__ grads, const float* __restrict__ binv,
                                            float* __restrict__ hb)
{
    const int ch = threadIdx.x;
    if (ch >= 3) return;
    const BnDesc d = desc[ch < 2 ? pol_layer : val_layer];
    const int c = ch < 2 ? ch : 0;
    const double N = (double)B * PIX;
    double s = 0.0, q = 0.0;
    for (int k = 0; k < HSC; ++k) {
        s += part[(ch * HSC + k) * 2 + 0];
        q += part[(ch * HSC + k) * 2 + 1];
    }
    const float inv = binv[d.out_off + c];
    const double invd = (double)inv;
    grads[d.gamma_off + c] = (float)(q * invd);
    grads[d.beta_off + c] = (float)s;
    hb[ch * 3 + 0] = (float)(s / N);
    hb[ch * 3 + 1] = (float)(q * invd * invd / N);
    hb[ch * 3 + 2] = inv * params[d.gamma_off + c];
}

__global__ __launch_bounds__(256) void head_bn_bwd_apply_kernel(const float* __restrict__ zh,
                                                                const float* __restrict__ dfp,
                                                                const float* __restrict__ dfv,
                                                                const float* __restrict__ hmean,
                                                                const float* __restrict__ hb, float* __restrict__ dzh,
                                                                int B)
{
    const int total = B * 3 * PIX;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int b = i / (3 * PIX), k = i - b * 3 * PIX;
        const int ch = k / PIX, p = k - ch * PIX;
        const float dy = ch < 2 ? dfp[(size_t)b * 2 * PIX + k] : dfv[(size_t)b * PIX + p];
        dzh[i] = ((dy - hb[ch * 3 + 0]) - (zh[i] - hmean[ch]) * hb[ch * 3 + 1]) * hb[ch * 3 + 2];
    }
}

// gX[m][c] = S_ch dzh[m][ch] * Wh[ch][c]; partial S_m dzh[m][ch] X[m][c] per tile
template <int C>
__global__ __launch_bounds__(256) void heads_bwd_proj_kernel(const float* __restrict__ act,
                                                             const float* __restrict__ dzh,
                                                             const float* __restrict__ wpc,
                                                             const float* __restrict__ wvc,
                                                             float* __restrict__ gx, float* __restrict__ hpart,
                                                             int M)
{
    // float4 over channels (C/4 threads per pixel row, 256*4/C rows per pass, 4 rows
    // in flight per thread); the per-thread partial sums of the three 1x1-conv weight
    // grads are added over the row groups in fixed order
    constexpr int Q = C / 4, RG = 256 / Q, UNR = 4;
    __shared__ f32x4 red[3][RG][Q];
    const int q = threadIdx.x % Q, rg = threadIdx.x / Q;
    const int c = 4 * q;
    const int m0 = blockIdx.x * HROWS;
    const int rows = min(HROWS, M - m0);
    const f32x4 w0 = *(const f32x4*)(wpc + c), w1 = *(const f32x4*)(wpc + C + c), w2 = *(const f32x4*)(wvc + c);
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0;
    for (int r0 = rg; r0 < rows; r0 += RG * UNR) {
        f32x4 xv[UNR];
        float d0[UNR], d1[UNR], d2[UNR];
        int o[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int r = r0 + RG * u;
            const int m = m0 + min(r, rows - 1);
            const int b = m / PIX, p = m - b * PIX;
            d0[u] = dzh[(b * 3 + 0) * PIX + p];
            d1[u] = dzh[(b * 3 + 1) * PIX + p];
            d2[u] = dzh[(b * 3 + 2) * PIX + p];
            o[u] = pad_off(m, C) + c;
            xv[u] = *(const f32x4*)(act + o[u]);
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
                }
                *(f32x4*)(gx + o[u]) = g;
            }
        }
    }
    red[0][rg][q] = s0;
    red[1][rg][q] = s1;
    red[2][rg][q] = s2;
    __syncthreads();
    if (rg == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            f32x4 a = red[k][0][q];
            for (int g = 1; g < RG; ++g) a += red[k][g][q];
            *(f32x4*)(hpart + ((size_t)blockIdx.x * 3 + k) * C + c) = a;
        }
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
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const double* __restrict__ part, int nb, float max_norm,
                                                   float* __restrict__ scal, float* __restrict__ total_norm,
                                                   float lr_bc1, float b1w, float b2, float one_m_b2, float bc2_sqrt,
                                                   float eps, float wd)
{
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
    A(w->DZ, act, true);
    A(w->DH, act, true);
    A(w->GR, act, true);
    A(w->DZ2, act, true);
    w->dzs.assign(2 * NB, nullptr);
    for (int k = 0; k < 2 * NB; ++k) A(w->dzs[k], act, true);

    {
        // the weight grads are off the critical path: their stream gets the LOWEST
        // priority so the dependent chain on the caller's stream (BN kernels, dgrad)
        // is dispatched first whenever workgroup slots free up
        hipError_t e = make_side_stream(w);
        if (e == hipSuccess) e = make_events(w);
        if (e != hipSuccess) return set_error("train: side stream / events", e);
    }
    A(w->wdpack, (size_t)(2 * NB > 0 ? 2 * NB : 1) * 9 * C * C, false);
    const size_t nf = h->nfold;
    A(w->bmean, nf, true); A(w->binv, nf, true); A(w->bscale, nf, true); A(w->bshift, nf, true);
    A(w->bgm, nf, true); A(w->bk, nf, true); A(w->biw, nf, true);
    A(w->part_a, (size_t)ntile * C, false);
    A(w->part_b, (size_t)ntile * C, false);
    A(w->hpart, (size_t)((M + HROWS - 1) / HROWS) * 3 * C, false);
    A(w->spart, (size_t)cap * STEM_WG_CHUNKS * 27 * C, false);
    // split-K for wgrad: ~512 rows per split
    w->S = kMaxWgradSplits;
    A(w->slab, (size_t)w->S * 9 * C * C, false);
    A(w->slab2, (size_t)w->S * 9 * C * C, false);
    A(w->gslab[0], (size_t)8 * 9 * C * C, false);
    A(w->gslab[1], (size_t)8 * 9 * C * C, false);
    {
        float* gc = nullptr;
        A(gc, 9 * 16 * 8, true);   // 9 taps x (C/128)^2 tiles x 8 groups, C <= 512
        w->gcnt = (unsigned*)gc;
    }
    A(w->zh, (size_t)cap * 3 * PIX, false);
    A(w->fp, (size_t)cap * 2 * PIX, false);
    A(w->fv, (size_t)cap * PIX, false);
    A(w->hv, (size_t)cap * VHID, false);
    A(w->dpre, (size_t)cap, false);
    A(w->dlogits, (size_t)cap * ACTIONS, false);
    A(w->dfp, (size_t)cap * 2 * PIX, false);
    A(w->dfv, (size_t)cap * PIX, false);
    A(w->dhv, (size_t)cap * VHID, false);
    A(w->dzh, (size_t)cap * 3 * PIX, false);
    A(w->lossb, (size_t)cap * 2, false);
    A(w->lpre, (size_t)cap * ACTIONS, false);
    A(w->hpre, (size_t)cap * VHID, false);
    A(w->hbw, 16, false);
    {
        float* hp = nullptr;
        A(hp, 3 * HSC * 2 * 2, false);
        w->hspart = (double*)hp;
    }
    float* np = nullptr;
    A(np, 2 * 1024, false);
    w->npart = (double*)np;
    A(w->scal, 4, true);
    {
        float* fc = nullptr;
        A(fc, 64, true);
        w->fincnt = (unsigned*)fc;
        float* hc = nullptr;
        A(hc, 16, true);
        w->hcnt = (unsigned*)hc;
        float* t = nullptr;
        A(t, (size_t)head_proj_stats_groups(M) * 6 * 2, false);
        w->hsp1 = (double*)t;
        A(t, (size_t)head_board_groups(cap) * head_board_pd() * 2, false);
        w->hpd = (double*)t;
        A(w->hpf, (size_t)head_board_groups(cap) * head_board_pf(), false);
        A(t, (size_t)head_dgrad_groups(cap) * 6 * 2, false);
        w->hdp = (double*)t;
        A(w->feat, (size_t)cap * FC_FS, true);
        A(w->pre, (size_t)cap * FC_OUT, false);
    }
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

int g_wgrad_serial = 0;   // 1: conv weight grads on the caller's stream (A/B timing)
int g_train_fuse_apply = 1;   // key 23: 1 BN applies folded into the next conv's staging; 0 separate passes
int g_train_fuse_fin = 1;     // key 24: 1 BN finalize by the last workgroup of the producing conv; 0 separate kernels
int g_train_skip = 0;     // study build only (key 19): skip BN kernels to time them in situ (results invalid)
int g_train_split_pack = 1;   // key 30: 1 split repack (stem on the stream, the rest on the side stream); 0 one launch
int g_train_maskz = 1;   // key 29: 1 BN-backward apply of residual-free layers forms its ReLU mask from z (default); 0 reads act
int g_train_fuse_heads = 28;   // key 28: bit mask of the fused head stages (pv_train_heads.hip); 0 the 18-launch chain
int g_train_side_heads = 1;   // key 32: 1 the head weight-grad work deferred to the end of the tower backward; 0 in the head chain

template <int C>
static int32_t train_backward_t(azg_pv* h, const float* x, const float* pis, const float* zs, int B,
                                float* losses, hipStream_t st)
{
    TrainWS* w = ws_of(h);
    const int NB = h->NB;
    const int M = B * PIX;
    const int ntile = (M + TROWS - 1) / TROWS;
    const float* P = h->params;
    float* G = h->grads;
    const BnDesc* bd = h->bn_desc.data();
    const BnDesc* bdd = (const BnDesc*)h->bn_desc_dev;
    const int gM = grid_for((int64_t)M * C / 4);

    const int ntt = (M + TRAIN_BM - 1) / TRAIN_BM;   // M tiles of conv3x3_train (partials per tile)
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
        if (g_train_skip & 2) return 0;
        hipLaunchKernelGGL(bn_fin_tiles_kernel<true>, dim3((bd[layer].c + 63) / 64), dim3(512), 0, st, w->part_a,
                           w->part_b, nt, prow, M, C, bd[layer].c, fin_args(layer, true));
        AZG_CK(hipGetLastError(), "train: bn_finalize_tiles");
        return 0;
    };
    // the conv3x3_train launch that produces a layer's partials also finalizes it
    // (key 24; the fused and the separate finalize are bitwise identical)
    const bool ffin = g_train_fuse_fin != 0 && !(g_train_skip & 10);
    // stem: separate column statistics (64-row tiles)
    auto stats = [&](const float* z, int layer) -> int32_t {
        int pr = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
        hipLaunchKernelGGL((col_stats_kernel<C>), dim3(ntile), dim3(256), 0, st, z, w->part_a, w->part_b, M);
        AZG_CK(hipGetLastError(), "train: col_stats");
        if (int32_t r = fin_fwd(layer, TROWS, ntile)) return r;
        prof_end(h, pr, st);
        return 0;
    };
    auto apply = [&](const float* z, const float* res, int layer, float* out) -> int32_t {
        if (g_train_skip & 1) return 0;
        const int o = bd[layer].out_off;
        const bool wt = (g_train_wt & 2) != 0;
        if (res && wt)
            hipLaunchKernelGGL((bn_apply_kernel<C, true, true>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        else if (res)
            hipLaunchKernelGGL((bn_apply_kernel<C, true>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        else if (wt)
            hipLaunchKernelGGL((bn_apply_kernel<C, false, true>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        else
            hipLaunchKernelGGL((bn_apply_kernel<C, false>), dim3(gM), dim3(256), 0, st, z, res, w->bscale + o,
                               w->bshift + o, out, M);
        AZG_CK(hipGetLastError(), "train: bn_apply");
        return 0;
    };
    // train-mode conv: forward (z + BN tile statistics) or dgrad (+ BN-backward tile
    // sums of the layer below: act / z / layer `xl`); partials land in part_a / part_b
    // fin >= 0: the BN layer this launch's partials belong to, finalized in-kernel
    auto conv = [&](int epi, int xe, const float* in, const float* wp, const float* res, float* out,
                    const float* xact, const float* xz, int xl, int fin = -1) -> int32_t {
        int pr = prof_begin(h, AZG_PROF_TRAIN_CONV, st, B);
        const EpiX ex{xact, xz, xl >= 0 ? w->bmean + bd[xl].out_off : nullptr, w->part_a, w->part_b};
        FinX fx{};
        if (fin >= 0) {
            fx = fin_args(fin, xe == XE_STATS);
            fx.cnt = w->fincnt;
            fx.late = xe == XE_STATS ? g_train_late_store : 0;
        }
        AZG_CK(launch_conv3x3_train(C, epi, xe, in, wp, res, out, M, ex, st, nullptr, fin >= 0 ? &fx : nullptr),
               "train: conv3x3");
        prof_end(h, pr, st);
        return 0;
    };
    auto bwd_reduce = [&](const float* g, const float* act, const float* z, int layer) -> int32_t {
        hipLaunchKernelGGL((bn_bwd_reduce_kernel<C>), dim3(ntile), dim3(256), 0, st, g, act, z,
                           w->bmean + bd[layer].out_off, w->part_a, w->part_b, M);
        AZG_CK(hipGetLastError(), "train: bn_bwd_reduce");
        return 0;
    };
    auto bwd_fin = [&](int layer, int nt) -> int32_t {
        if (g_train_skip & 8) return 0;
        hipLaunchKernelGGL(bn_fin_tiles_kernel<false>, dim3((bd[layer].c + 63) / 64), dim3(512), 0, st,
                           w->part_a, w->part_b, nt, 1, M, C, bd[layer].c, fin_args(layer, false));
        AZG_CK(hipGetLastError(), "train: bn_bwd_finalize_tiles");
        return 0;
    };
    // mz: the layer has no residual input -- its ReLU mask comes from z (bn_bwd_apply MZ)
    auto bwd_apply = [&](const float* g, const float* act, const float* z, int layer, float* dz,
                         float* gres, bool mz = false) -> int32_t {
        if (g_train_skip & 4) return 0;
        const int o = bd[layer].out_off;
        const bool wt = (g_train_wt & 2) != 0;
        mz = mz && g_train_maskz;
#define AZG_BWD_APPLY(GR, W, MZ)                                                                              \
        hipLaunchKernelGGL((bn_bwd_apply_kernel<C, GR, W, MZ>), dim3(gM), dim3(256), 0, st, g, act, z,        \
                           w->bmean + o, w->bgm + o, w->bk + o, w->biw + o, dz, gres, M, w->bscale + o,         \
                           w->bshift + o)
        if (gres && wt) AZG_BWD_APPLY(true, true, false);
        else if (gres) AZG_BWD_APPLY(true, false, false);
        else if (wt && mz) AZG_BWD_APPLY(false, true, true);
        else if (wt) AZG_BWD_APPLY(false, true, false);
        else if (mz) AZG_BWD_APPLY(false, false, true);
        else AZG_BWD_APPLY(false, false, false);
#undef AZG_BWD_APPLY
        AZG_CK(hipGetLastError(), "train: bn_bwd_apply");
        return 0;
    };
    // weight gradient of one conv on the side stream, after dZ is ready
    bool pending[2] = {false, false};
    float* dzbuf[2] = {w->DZ, w->DZ2};
    const bool dz_all = g_train_dz_all != 0 && !g_wgrad_serial;
    bool side_used = false;
    // key 39: a weight grad's slab reduction is launched on `side` after the NEXT conv's
    // weight-grad kernel (two alternating slab buffers), so each weight-grad kernel starts
    // as soon as its dZ is ready, ahead of the previous reduction's HBM pass
    const bool defer_red = g_train_defer_reduce != 0 && !g_wgrad_serial;
    // key 39 = 2: the step's last weight grad leaves its own and the previous conv's
    // reductions pending; both run in one launch on the caller's stream after the join
    // (idle there, while `side` would run them back to back ahead of the join)
    const bool tail_red = defer_red && g_train_defer_reduce == 2;
    struct PendRed { float* slab; float* dw; int S; };
    PendRed pend_red{nullptr, nullptr, 0}, pend_red2{nullptr, nullptr, 0};
    float* slabs[2] = {w->slab, w->slab2};
    int slab_i = 0;
    auto flush_red = [&]() -> int32_t {
        if (pend_red.slab) AZG_CK(launch_wgrad_reduce(C, pend_red.slab, pend_red.dw, pend_red.S, w->side),
                                  "train: wgrad reduce");
        pend_red = PendRed{nullptr, nullptr, 0};
        return 0;
    };
    // dZ of backward conv k (2i+1: conv2 of block i, 2i: conv1): its own buffer (key 34)
    // or the alternating slot
    auto dzb = [&](int k, int slot) -> float* { return dz_all ? w->dzs[k] : dzbuf[slot]; };
    auto wgrad = [&](int slot, const float* dz, const float* xin, int tensor, bool last = false) -> int32_t {
        if (g_wgrad_serial) {   // A/B: weight grads on the caller's stream, no overlap
            int pr = prof_begin(h, AZG_PROF_TRAIN_WGRAD, st);
            const int S = wgrad_splits(C, M);
            if (S > w->S) return set_error("train: wgrad splits exceed the slab workspace", hipErrorInvalidValue);
            AZG_CK(launch_wgrad(C, dz, xin, w->slab, G + h->poff[tensor], M, S, st, true, w->gcnt, w->gslab[0]),
                   "train: wgrad");
            prof_end(h, pr, st);
            return 0;
        }
        AZG_CK(hipEventRecord(w->ev_ready[slot], st), "train: event record");
        AZG_CK(hipStreamWaitEvent(w->side, w->ev_ready[slot], 0), "train: stream wait");
        int pr = prof_begin(h, AZG_PROF_TRAIN_WGRAD, w->side);
        const int S = wgrad_splits(C, M);
        if (S > w->S) return set_error("train: wgrad splits exceed the slab workspace", hipErrorInvalidValue);
        float* sl = defer_red ? slabs[slab_i] : w->slab;
        const bool comb = wgrad_comb_on(g_wgrad_kernel, S);
        float* gsl = w->gslab[defer_red ? slab_i : 0];
        AZG_CK(launch_wgrad(C, dz, xin, sl, G + h->poff[tensor], M, S, w->side, !defer_red, w->gcnt, gsl),
               "train: wgrad");
        if (defer_red) {   // the previous conv's reduction behind this conv's MFMA work
            if (tail_red && last) pend_red2 = pend_red;   // to the caller's stream after the join
            else if (int32_t r2 = flush_red()) return r2;
            pend_red = comb ? PendRed{gsl, G + h->poff[tensor], 8} : PendRed{sl, G + h->poff[tensor], S};
            slab_i ^= 1;
        }
        prof_end(h, pr, w->side);
        side_used = true;
        if (!dz_all) {
            AZG_CK(hipEventRecord(w->ev_done[slot], w->side), "train: event record");
            pending[slot] = true;
        }
        return 0;
    };
    // the caller's stream may overwrite dZ (slot) only after its wgrad has read it
    auto reuse = [&](int slot) -> int32_t {
        if (pending[slot]) {
            AZG_CK(hipStreamWaitEvent(st, w->ev_done[slot], 0), "train: stream wait");
            pending[slot] = false;
        }
        return 0;
    };
    int32_t r;
#define R(x) if ((r = (x))) return r

    // ---- forward (train-mode BN) ----
    bool last_apply = false;   // the last block's BN apply is left to the fused head kernel
    struct LastApply { const float* z; const float* res; int layer; float* out; } lastp{nullptr, nullptr, 0, nullptr};
    if (g_train_stem_stats && !(g_train_skip & 2)) {
        int pr0 = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
        AZG_CK(launch_stem_stats(C, x, h->wstem, w->z0, B, w->part_a, w->part_b, st), "train: stem + statistics");
        R(fin_fwd(h->bn_stem, 128, (M + 127) / 128));
        prof_end(h, pr0, st);
    } else {
        AZG_CK(launch_stem(C, EPI_RAW, x, h->wstem, nullptr, nullptr, w->z0, B, st), "train: stem");
        R(stats(w->z0, h->bn_stem));
    }
    if (w->pack_pending) {   // the residual convs' packs (split repack, train_backward)
        AZG_CK(hipStreamWaitEvent(st, w->ev_pack, 0), "train: stream wait");
        w->pack_pending = false;
    }
    const float* X = w->a0;
    // the staging prologue fits the 128-VGPR tile body at C <= 128; at C = 256 (eight
    // channel groups unrolled) it spills 96 VGPRs and costs ~1 ms per 10x256 step
    // (measured), so the separate apply passes stay there
    if (g_train_fuse_apply && C <= 128) {
        // every BN apply but the last is done by the next conv's halo staging
        // (pv_halo.h ProX): `pend` = the activation still to be formed from its raw z
        struct Pend { const float* z; int layer; const float* res; float* out; };
        Pend pend{w->z0, h->bn_stem, nullptr, w->a0};
        auto fused_conv = [&](const Pend& p, const float* wpk, float* out, int fin) -> int32_t {
            int pr = prof_begin(h, AZG_PROF_TRAIN_CONV, st, B);
            const int o = bd[p.layer].out_off;
            const EpiX ex{nullptr, nullptr, nullptr, w->part_a, w->part_b};
            const ProX px{p.res, w->bscale + o, w->bshift + o, p.out};
            FinX fx = fin_args(fin, true);
            fx.cnt = w->fincnt;
            fx.late = g_train_late_store;
            AZG_CK(launch_conv3x3_train(C, EPI_RAW, XE_STATS, p.z, wpk, nullptr, out, M, ex, st, &px,
                                        ffin ? &fx : nullptr),
                   "train: conv3x3 (fused BN apply)");
            prof_end(h, pr, st);
            if (!ffin) return fin_fwd(fin, TRAIN_BM, ntt);
            return 0;
        };
        for (int i = 0; i < NB; ++i) {
            R(fused_conv(pend, h->wpack + (size_t)(2 * i) * 9 * C * C, w->z1[i], h->bn_blk[i].first));
            pend = Pend{w->z1[i], h->bn_blk[i].first, nullptr, w->hh[i]};
            R(fused_conv(pend, h->wpack + (size_t)(2 * i + 1) * 9 * C * C, w->z2[i], h->bn_blk[i].second));
            pend = Pend{w->z2[i], h->bn_blk[i].second, X, w->xo[i]};
            X = w->xo[i];
        }
        if ((g_train_fuse_heads & 17) && pend.res) {
            last_apply = true;   // the head kernel applies bn2 + residual + ReLU of the last block
            lastp = {pend.z, pend.res, pend.layer, pend.out};
        } else {
            R(apply(pend.z, pend.res, pend.layer, pend.out));
        }
    } else {
        R(apply(w->z0, nullptr, h->bn_stem, w->a0));
        for (int i = 0; i < NB; ++i) {
            const int l1 = h->bn_blk[i].first, l2 = h->bn_blk[i].second;
            R(conv(EPI_RAW, XE_STATS, X, h->wpack + (size_t)(2 * i) * 9 * C * C, nullptr, w->z1[i], nullptr, nullptr,
                   -1, ffin ? l1 : -1));
            if (!ffin) R(fin_fwd(l1, TRAIN_BM, ntt));
            R(apply(w->z1[i], nullptr, l1, w->hh[i]));
            R(conv(EPI_RAW, XE_STATS, w->hh[i], h->wpack + (size_t)(2 * i + 1) * 9 * C * C, nullptr, w->z2[i],
                   nullptr, nullptr, -1, ffin ? l2 : -1));
            if (!ffin) R(fin_fwd(l2, TRAIN_BM, ntt));
            R(apply(w->z2[i], X, h->bn_blk[i].second, w->xo[i]));
            X = w->xo[i];
        }
    }
    // ---- heads forward + loss + backward to the tower output ----
    // key 28 bit 0: head 1x1 projections + BN statistics + finalize in one launch
    // (head_proj_stats, also applying the last block's bn2 + residual + ReLU); bit 1: head
    // BN apply + FCs + loss + fc data grads + head BN-backward sums in one launch per 4
    // boards (head_board); bit 2: head BN-backward apply + 1x1 data/weight-grad partials +
    // the last block's BN-backward partials in one launch (heads_bwd_fused)
    const int hntile = (M + HROWS - 1) / HROWS;
    const int fh = g_train_fuse_heads;
    const int ho = bd[h->bn_pol].out_off;   // policy ch0, ch1, value: contiguous
    const float* wpf = P + h->poff[h->t_pfc_w];
    const float* wv1 = P + h->poff[h->t_vfc1_w];
    int pr = prof_begin(h, AZG_PROF_TRAIN_OTHER, st);
    // key 28 bits 3 + 4: both head finalizes folded into their consumer kernels
    const bool fold_fin = (fh & 8) && (fh & 16);
    HeadStatsArgs hs{};
    HeadDgradArgs hd{};
    if (fh & 17) {
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
        hs.cnt = w->hcnt;
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
        if (fold_fin) AZG_CK(launch_head_proj_partials(C, last_apply, hs, st), "train: head_proj_partials");
        else if (fh & 16) AZG_CK(launch_head_proj_split(C, last_apply, hs, st), "train: head_proj_split");
        else AZG_CK(launch_head_proj_stats(C, last_apply, hs, st), "train: head_proj_stats");
    } else {
        AZG_CK(launch_heads_project(C, false, X, P + h->poff[h->t_pc_w], P + h->poff[h->t_vc_w], nullptr, nullptr,
                                    w->zh, M, st),
               "train: heads_project");
        hipLaunchKernelGGL(head_stats_partial_kernel, dim3(3, HSC), dim3(256), 0, st, w->zh, B, w->hspart);
        AZG_CK(hipGetLastError(), "train: head_stats_partial");
        hipLaunchKernelGGL(head_stats_finalize_kernel, dim3(1), dim3(64), 0, st, w->hspart, B, bdd, h->bn_pol,
                           h->bn_val, P, h->bn, w->bmean, w->binv, w->bscale, w->bshift, h->nbt,
                           (int)h->bn_desc.size());
        AZG_CK(hipGetLastError(), "train: head_stats_finalize");
    }
    const int gH = grid_for((int64_t)B * 3 * PIX);
    // head weight-grad work only Adam reads waits for the end of the tower backward (key
    // 32): the side stream is the backward's bottleneck (it ends after the caller's),
    // while the caller's stream idles there
    const bool defer_heads = g_train_side_heads == 1 && (fh & 8);
    const bool side_heads = g_train_side_heads == 2 && (fh & 8) && !g_wgrad_serial;   // on `side` during the head chain
    // the fc weight grads, their biases / value_fc2 and the loss means (key 28 bit 3)
    auto fc_wgrads = [&](hipStream_t ws) -> int32_t {
        // weight grads: dWpf = dlogits^T . fp, dWv1 = dhv^T . fv
        AZG_CK(launch_head_fc_wgrad(w->dlogits, w->fp, w->dhv, w->fv, G + h->poff[h->t_pfc_w], G + h->poff[h->t_vfc1_w],
                                    B, ws),
               "train: head fc wgrad");
        hipLaunchKernelGGL(heads_small_grads_kernel, dim3((HSG_OUT + 3) / 4), dim3(256), 0, ws, w->dlogits, w->dhv,
                           w->dpre, w->hv, w->lossb, B, G + h->poff[h->t_pfc_b], G + h->poff[h->t_vfc1_b],
                           G + h->poff[h->t_vfc2_w], G + h->poff[h->t_vfc2_b], losses);
        AZG_CK(hipGetLastError(), "train: heads_small_grads");
        return 0;
    };
    if (fh & 8) {
        // short, wide launches: features in the eval row layout -> heads_fc (MFMA) ->
        // heads_loss -> masked fc dgrad + head-BN backward partials -> one-wave finalize;
        // the weight grads of the fcs and their biases / value_fc2 (and the loss means) on
        // the side stream
        AZG_CK(launch_head_bn_apply_feat(w->zh, w->bscale + ho, w->bshift + ho, w->fp, w->fv, w->feat, B, st,
                                         fold_fin ? &hs : nullptr),
               "train: head_bn_apply_feat");
        AZG_CK(launch_heads_fc(w->feat, h->wfc, w->pre, B, st), "train: heads_fc");
        hipLaunchKernelGGL(heads_loss_kernel, dim3((B + 3) / 4), dim3(256), 0, st, w->pre, P + h->poff[h->t_pfc_b],
                           w->pre + ACTIONS, P + h->poff[h->t_vfc1_b], P + h->poff[h->t_vfc2_w],
                           P + h->poff[h->t_vfc2_b], pis, zs, w->dlogits, w->hv, w->dhv, w->dpre, w->lossb, B,
                           FC_OUT, FC_OUT);
        AZG_CK(hipGetLastError(), "train: heads_loss");
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
        hd.hb = w->hbw;
        if (side_heads) {   // the fc weight grads only need the loss stage: run them on the idle side stream
            AZG_CK(hipEventRecord(w->ev_ready[0], st), "train: event record");
            AZG_CK(hipStreamWaitEvent(w->side, w->ev_ready[0], 0), "train: stream wait");
            R(fc_wgrads(w->side));
            side_used = true;
        }
        AZG_CK(launch_head_dgrad(hd, st, !fold_fin), "train: head_dgrad");
        if (!defer_heads && !side_heads) R(fc_wgrads(st));   // else after the tower backward / on `side`
    } else if (fh & 2) {
        HeadBoardArgs hb{};
        hb.zh = w->zh;
        hb.hmean = w->bmean + ho;
        hb.hscale = w->bscale + ho;
        hb.hshift = w->bshift + ho;
        hb.hinv = w->binv + ho;
        hb.wfc = h->wfc;   // packed by this step's repack
        hb.wpf = wpf;
        hb.bpf = P + h->poff[h->t_pfc_b];
        hb.wv1 = wv1;
        hb.bv1 = P + h->poff[h->t_vfc1_b];
        hb.wv2 = P + h->poff[h->t_vfc2_w];
        hb.bv2 = P + h->poff[h->t_vfc2_b];
        hb.pis = pis;
        hb.zs = zs;
        hb.fp = w->fp;
        hb.fv = w->fv;
        hb.hv = w->hv;
        hb.dlogits = w->dlogits;
        hb.dhv = w->dhv;
        hb.dfp = w->dfp;
        hb.dfv = w->dfv;
        hb.pd = w->hpd;
        hb.pf = w->hpf;
        hb.cnt = w->hcnt + 1;
        hb.B = B;
        hb.desc = bdd;
        hb.pol_layer = h->bn_pol;
        hb.val_layer = h->bn_val;
        hb.params = P;
        hb.grads = G;
        hb.hb = w->hbw;
        hb.g_pfb = G + h->poff[h->t_pfc_b];
        hb.g_v1b = G + h->poff[h->t_vfc1_b];
        hb.g_v2w = G + h->poff[h->t_vfc2_w];
        hb.g_v2b = G + h->poff[h->t_vfc2_b];
        hb.losses = losses;
        AZG_CK(launch_head_board(hb, st), "train: head_board");
        {   // weight grads: dWpf = dlogits^T . fp, dWv1 = dhv^T . fv
            GemmProb a{w->dlogits, 1, ACTIONS, w->fp, 2 * PIX, 1, G + h->poff[h->t_pfc_w], 2 * PIX, 1, nullptr, 0, 0,
                       ACTIONS, 2 * PIX, B};
            GemmProb b{w->dhv, 1, VHID, w->fv, PIX, 1, G + h->poff[h->t_vfc1_w], PIX, 1, nullptr, 0, 0, VHID, PIX, B};
            AZG_CK(launch_small_gemm(a, &b, st), "train: head fc wgrad");
        }
    } else {
        hipLaunchKernelGGL(head_bn_apply_kernel, dim3(gH), dim3(256), 0, st, w->zh, w->bscale + ho, w->bshift + ho,
                           w->fp, w->fv, B);
        AZG_CK(hipGetLastError(), "train: head_bn_apply");
        {   // logits / value hidden pre-activations
            GemmProb a{w->fp, 2 * PIX, 1, wpf, 1, 2 * PIX, w->lpre, ACTIONS, 1, nullptr, 0, 0, B, ACTIONS, 2 * PIX};
            GemmProb b{w->fv, PIX, 1, wv1, 1, PIX, w->hpre, VHID, 1, nullptr, 0, 0, B, VHID, PIX};
            AZG_CK(launch_small_gemm(a, &b, st), "train: head fc fwd");
        }
        hipLaunchKernelGGL(heads_loss_kernel, dim3((B + 3) / 4), dim3(256), 0, st, w->lpre, P + h->poff[h->t_pfc_b],
                           w->hpre, P + h->poff[h->t_vfc1_b], P + h->poff[h->t_vfc2_w], P + h->poff[h->t_vfc2_b],
                           pis, zs, w->dlogits, w->hv, w->dhv, w->dpre, w->lossb, B);
        AZG_CK(hipGetLastError(), "train: heads_loss");
        {   // dfp = (dlogits . Wpf) * (fp > 0), dfv = (dhv . Wv1) * (fv > 0)
            GemmProb a{w->dlogits, ACTIONS, 1, wpf, 2 * PIX, 1, w->dfp, 2 * PIX, 1, w->fp, 2 * PIX, 1, B, 2 * PIX,
                       ACTIONS};
            GemmProb b{w->dhv, VHID, 1, wv1, PIX, 1, w->dfv, PIX, 1, w->fv, PIX, 1, B, PIX, VHID};
            AZG_CK(launch_small_gemm(a, &b, st), "train: head fc dgrad");
        }
        {   // weight grads: dWpf = dlogits^T . fp, dWv1 = dhv^T . fv
            GemmProb a{w->dlogits, 1, ACTIONS, w->fp, 2 * PIX, 1, G + h->poff[h->t_pfc_w], 2 * PIX, 1, nullptr, 0, 0,
                       ACTIONS, 2 * PIX, B};
            GemmProb b{w->dhv, 1, VHID, w->fv, PIX, 1, G + h->poff[h->t_vfc1_w], PIX, 1, nullptr, 0, 0, VHID, PIX, B};
            AZG_CK(launch_small_gemm(a, &b, st), "train: head fc wgrad");
        }
        hipLaunchKernelGGL(heads_small_grads_kernel, dim3((HSG_OUT + 3) / 4), dim3(256), 0, st, w->dlogits, w->dhv,
                           w->dpre, w->hv, w->lossb, B, G + h->poff[h->t_pfc_b], G + h->poff[h->t_vfc1_b],
                           G + h->poff[h->t_vfc2_w], G + h->poff[h->t_vfc2_b], losses);
        AZG_CK(hipGetLastError(), "train: heads_small_grads");
        hipLaunchKernelGGL(head_bn_bwd_partial_kernel, dim3(3, HSC), dim3(256), 0, st, w->zh, w->dfp, w->dfv, B,
                           w->bmean + ho, w->hspart);
        AZG_CK(hipGetLastError(), "train: head_bn_bwd_partial");
        hipLaunchKernelGGL(head_bn_bwd_finalize_kernel, dim3(1), dim3(64), 0, st, w->hspart, B, bdd, h->bn_pol,
                           h->bn_val, P, G, w->binv, w->hbw);
        AZG_CK(hipGetLastError(), "train: head_bn_bwd_finalize");
    }
    if (fh & 4) {
        HeadBwdArgs hw{};
        hw.act = X;
        hw.zh = w->zh;
        hw.dfp = w->dfp;
        hw.dfv = w->dfv;
        hw.hmean = w->bmean + ho;
        hw.hb = w->hbw;
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
        if (fold_fin) {
            hw.dg = hd;
            hw.dg_nwg = head_dgrad_groups(B);
        }
        AZG_CK(launch_heads_bwd_fused(C, NB > 0, hw, st), "train: heads_bwd_fused");
    } else {
        hipLaunchKernelGGL(head_bn_bwd_apply_kernel, dim3(gH), dim3(256), 0, st, w->zh, w->dfp, w->dfv, w->bmean + ho,
                           w->hbw, w->dzh, B);
        AZG_CK(hipGetLastError(), "train: head_bn_bwd_apply");
        hipLaunchKernelGGL((heads_bwd_proj_kernel<C>), dim3(hntile), dim3(256), 0, st, X, w->dzh,
                           P + h->poff[h->t_pc_w], P + h->poff[h->t_vc_w], w->gX, w->hpart, M);
        AZG_CK(hipGetLastError(), "train: heads_bwd_proj");
    }
    // policy_conv.weight [2][C] then value_conv.weight [C]: partial layout [t][3][C]
    auto head_proj_wgrad = [&]() -> int32_t {
        hipLaunchKernelGGL(reduce_partials_kernel, dim3((3 * C + 15) / 16), dim3(256), 0, st, w->hpart, hntile, 3 * C,
                           G + h->poff[h->t_pc_w], G + h->poff[h->t_vc_w], 2 * C, 0, C);
        AZG_CK(hipGetLastError(), "train: heads proj wgrad");
        return 0;
    };
    if (!defer_heads && !side_heads) R(head_proj_wgrad());
    prof_end(h, pr, st);
    auto snap = [&](int k) -> int32_t {
        if (!w->snap.empty())
            AZG_CK(hipMemcpyAsync(w->snap[k], w->gX, (size_t)B * PADPIX * C * sizeof(float), hipMemcpyDeviceToDevice, st),
                   "train: snapshot");
        return 0;
    };
    R(snap(0));
    // ---- tower backward ----
    // The BN-backward sums of every layer but the last block's bn2 come out of the
    // epilogue of the dgrad conv that produces its gradient (XE_BNBWD, per 128-row
    // tile); the last block's gradient comes from the heads (separate reduction).
    int bwd_nt = ntt;
    if (NB > 0 && (g_train_fuse_heads & 4)) {
        bwd_nt = hntile;   // S dy, S (z - mean) dy per 128-row tile from heads_bwd_fused_kernel
    } else if (NB > 0) {
        R(bwd_reduce(w->gX, w->xo[NB - 1], w->z2[NB - 1], h->bn_blk[NB - 1].second));
        bwd_nt = ntile;
    }
    // key 40: the dZ of each block's conv1 formed in its dgrad's staging (needs dz_all:
    // the weight grad reads dz1 after the dgrad; the bn1 mask from z1: key 29)
    const bool fuse_bwd = g_train_fuse_bwd && C <= 128 && dz_all && g_train_maskz && !(g_train_skip & 4);
    bool done_fin = false;   // the previous dgrad launch already finalized the next layer
    for (int i = NB - 1; i >= 0; --i) {
        const float* Xin = i == 0 ? w->a0 : w->xo[i - 1];
        const float* zin = i == 0 ? w->z0 : w->z2[i - 1];
        const int lin = i == 0 ? h->bn_stem : h->bn_blk[i - 1].second;
        if (!done_fin) R(bwd_fin(h->bn_blk[i].second, bwd_nt));
        R(reuse(0));
        float* dz2 = dzb(2 * i + 1, 0);
        R(bwd_apply(w->gX, w->xo[i], w->z2[i], h->bn_blk[i].second, dz2, w->GR));
        R(wgrad(0, dz2, w->hh[i], h->t_blk[i].w2));
        R(conv(EPI_RAW, XE_BNBWD, dz2, w->wdpack + (size_t)(2 * i + 1) * 9 * C * C, nullptr, w->DH, w->hh[i],
               w->z1[i], h->bn_blk[i].first, ffin ? h->bn_blk[i].first : -1));
        if (!ffin) R(bwd_fin(h->bn_blk[i].first, ntt));
        R(reuse(1));
        float* dz1 = dzb(2 * i, 1);
        if (fuse_bwd) {
            // bn1's backward (mask from z1, no residual) applied in this dgrad's staging;
            // its N-tile-0 workgroups write dz1 for the weight grad, which follows it
            const int o1 = bd[h->bn_blk[i].first].out_off;
            ProX px{w->z1[i], w->bscale + o1, w->bshift + o1, dz1, w->bmean + o1, w->bgm + o1, w->bk + o1, w->biw + o1};
            int pr = prof_begin(h, AZG_PROF_TRAIN_CONV, st, B);
            const EpiX ex{Xin, zin, w->bmean + bd[lin].out_off, w->part_a, w->part_b};
            FinX fx{};
            if (ffin) {
                fx = fin_args(lin, false);
                fx.cnt = w->fincnt;
                }
            AZG_CK(launch_conv3x3_train(C, EPI_ADD, XE_BNBWD, w->DH, w->wdpack + (size_t)(2 * i) * 9 * C * C, w->GR,
                                        w->gX, M, ex, st, &px, ffin ? &fx : nullptr),
                   "train: conv3x3 (fused BN backward)");
            prof_end(h, pr, st);
            R(wgrad(1, dz1, Xin, h->t_blk[i].w1, i == 0));
        } else {
            R(bwd_apply(w->DH, w->hh[i], w->z1[i], h->bn_blk[i].first, dz1, nullptr, true));
            R(wgrad(1, dz1, Xin, h->t_blk[i].w1, i == 0));
            R(conv(EPI_ADD, XE_BNBWD, dz1, w->wdpack + (size_t)(2 * i) * 9 * C * C, w->GR, w->gX, Xin, zin, lin,
                   ffin ? lin : -1));
        }
        done_fin = ffin;
        bwd_nt = ntt;
        R(snap(NB - i));
    }
    if (defer_red && !tail_red) R(flush_red());   // the last conv's reduction
    if (defer_heads) {   // the head weight grads (Adam's inputs only)
        R(fc_wgrads(st));
        R(head_proj_wgrad());
    } else if (side_heads) {
        R(head_proj_wgrad());
    }
    // ---- stem backward ----
    // overlaps the last conv weight grads still on the side stream: its dz goes to
    // DH (no pending weight grad reads DH), the join comes after it
    if (NB == 0) {
        R(bwd_reduce(w->gX, w->a0, w->z0, h->bn_stem));
        bwd_nt = ntile;
    }
    if (!done_fin) R(bwd_fin(h->bn_stem, bwd_nt));
    R(bwd_apply(w->gX, w->a0, w->z0, h->bn_stem, w->DH, nullptr, true));
    hipLaunchKernelGGL((stem_wgrad_kernel<C>), dim3(B * STEM_WG_CHUNKS), dim3(256), 0, st, x, w->DH, w->spart);
    AZG_CK(hipGetLastError(), "train: stem_wgrad");
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((27 * C + 15) / 16), dim3(256), 0, st, w->spart, B * STEM_WG_CHUNKS, 27 * C,
                       G + h->poff[h->t_stem_w], nullptr, 27 * C, 1, C);
    AZG_CK(hipGetLastError(), "train: stem_wgrad_reduce");
    R(reuse(0));
    R(reuse(1));                 // joins the side stream: every conv weight grad is done
    if (side_used) {             // (and the head weight grads when no conv weight grad follows them)
        AZG_CK(hipEventRecord(w->ev_join, w->side), "train: event record");
        AZG_CK(hipStreamWaitEvent(st, w->ev_join, 0), "train: stream wait");
    }
    if (tail_red && pend_red.slab) {   // key 39 = 2: the last two convs' reductions, one launch
        if (pend_red2.slab)
            AZG_CK(launch_wgrad_reduce2(C, pend_red2.slab, pend_red2.dw, pend_red2.S, pend_red.slab, pend_red.dw,
                                        pend_red.S, st),
                   "train: wgrad reduce (tail)");
        else
            AZG_CK(launch_wgrad_reduce(C, pend_red.slab, pend_red.dw, pend_red.S, st), "train: wgrad reduce (tail)");
        pend_red = pend_red2 = PendRed{nullptr, nullptr, 0};
    }
#undef R
    return 0;
}

int32_t train_backward(azg_pv* h, const float* x, const float* pis, const float* zs, int B, float* losses,
                       hipStream_t st)
{
    if (int32_t r = ensure_train_ws(h, B, st)) return r;
    TrainWS* w = ws_of(h);
    AZG_CK(make_side_stream(w), "train: side stream");
    AZG_CK(make_events(w), "train: events");
    if (h->train_packs) {
        // the packs were refreshed right after the last Adam step (train_apply, key 36) and
        // no parameter changed since (azg_pv_mark_dirty / bind clear the flag)
    } else if (g_train_split_pack && !g_wgrad_serial) {
        // the stem's pack on this stream; the residual convs' forward + dgrad packs and
        // the head FCs on the side stream, overlapping the stem and its statistics (the
        // first residual conv waits for them, train_backward_t)
        AZG_CK(hipEventRecord(w->ev_pack_in, st), "train: event record");
        AZG_CK(hipStreamWaitEvent(w->side, w->ev_pack_in, 0), "train: stream wait");
        if (int32_t r = repack(h, st, w->wdpack, 1)) return r;
        if (int32_t r = repack(h, w->side, w->wdpack, 2)) return r;
        AZG_CK(hipEventRecord(w->ev_pack, w->side), "train: event record");
        w->pack_pending = true;
    } else if (int32_t r = repack(h, st, w->wdpack)) {
        return r;
    }
    h->train_packs = true;
    const int C = h->C;
    int32_t r;
    switch (C) {
        case 64: r = train_backward_t<64>(h, x, pis, zs, B, losses, st); break;
        case 128: r = train_backward_t<128>(h, x, pis, zs, B, losses, st); break;
        case 256: r = train_backward_t<256>(h, x, pis, zs, B, losses, st); break;
        default: return set_error("train: bad channels", hipErrorInvalidValue);
    }
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
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n) < 1024 ? grid_for(n) : 1024), dim3(256), 0, st, h->params,
                       h->grads, exp_avg, exp_avg_sq, n, w->npart, nb, max_norm, w->scal, total_norm, lr_bc1,
                       (float)(1.0 - (double)beta1), beta2, (float)(1.0 - (double)beta2), bc2_sqrt, eps, wd);
    AZG_CK(hipGetLastError(), "apply: adam");
    h->train_packs = false;   // the parameters changed
    if (g_train_pack_after) {
        // every pack of the next step (and the eval BN fold) from the new parameters, on
        // this stream right behind Adam: the next train step starts without a repack and
        // without the cross-stream hand-off of the split repack (key 30)
        if (int32_t r = repack(h, st, w->wdpack)) return r;
        h->train_packs = true;
        h->dirty = false;
    } else {
        h->dirty = true;
    }
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
        case 7: src = (g_train_dz_all && !w->dzs.empty()) ? w->dzs[0] : w->DZ; break;   // the last backward conv's dZ
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
