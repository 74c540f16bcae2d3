// Halo-staged 3x3 conv tile (fp32 MFMA implicit GEMM), shared by the per-layer
// kernel (pv_conv.hip, conv3x3_halo) and the persistent residual-tower kernel
// (pv_tower.hip, conv_tower).  Replaces the ATen conv2d + batch_norm + relu
// (+ residual add) chain of the reference ResidualBlock (network.py:9-26).
//
// GEMM view: rows m = pixel of the batch (B*225), cols n = output channel,
// K = 9 taps x C input channels.  A[m][k] is read from the padded NHWC activation,
// B is the weight re-packed to [kchunk][n][32] (kchunk = tap*C/32 + cin/32) so a
// K-chunk of 32 is one contiguous block.
#pragma once
#include "pv_common.h"

#ifndef AZG_EVAL_REMAT
#define AZG_EVAL_REMAT 0   // study: 1 = per-tap addresses in the fp32 bodies too
#endif
namespace azg {

// Tile shape: BM = WM*TM*32 pixels x BN channels; NW waves as WM x WN (WN = NW/WM),
// each wave TM x TN accumulators of 32x32 (v_mfma_f32_32x32x2_f32: exact f32 FMA
// chain -- the parity budget is 1e-5 fp32, so no bf16).  Several shapes are
// compiled; the host picks by autotuning (all shapes are bitwise identical).
template <int C, int BN_, int WM_, int TM_, int NW_ = 4, int SB_ = 0>
struct ConvTile {
    static constexpr int NW = NW_;                // waves per workgroup
    static constexpr int NT = 64 * NW_;           // threads
    static constexpr int RPP = NT / 8;            // staging rows per pass (8 x 16 B per row)
    static constexpr int BN = BN_;
    static constexpr int WM = WM_;
    static constexpr int WN = NW_ / WM_;
    static constexpr int TM = TM_;
    static constexpr int TN = BN_ / (WN * 32);
    static constexpr int BM = WM * TM * 32;
    static constexpr int BK = 32;
    static constexpr int LDK = BK;          // unpadded rows; XOR-swizzled 16-B chunks
    static constexpr int CG = C / BK;
    static constexpr int NCH = 9 * CG;
    static constexpr int A_LD = BM * BK / 4 / NT;
    static constexpr int B_LD = BN * BK / 4 / NT;
    // SB_: single LDS buffer (the next chunk waits in registers; two barriers per
    // chunk) -- half the LDS per workgroup, twice the resident workgroups.
    static constexpr int LDS_BYTES = (SB_ ? 1 : 2) * (BM + BN) * LDK * 4;
    static_assert(TN >= 1 && WN * TN * 32 == BN, "bad tile");
    static_assert(A_LD >= 1 && B_LD >= 1 && A_LD * NT * 4 == BM * BK && B_LD * NT * 4 == BN * BK, "bad staging");
};

// Padded-pixel ("row") index of interior pixel m; a 3x3 tap is the constant row
// shift (ky-1)*17 + (kx-1).  Padded rows are contiguous across boards, so the
// input rows every tap of a BM-pixel tile reads form ONE contiguous range
// [row(m0) - 18, row(m0+BM-1) + 18]: the tile's halo.
__host__ __device__ constexpr int pad_row(int m)
{
    return (m / PIX) * PADPIX + ((m % PIX) / BOARD + 1) * PADW + (m % BOARD) + 1;
}
// largest halo (rows) over every tile position: m0 mod 225 repeats after 225 tiles
constexpr int halo_span(int BM)
{
    int mx = 0;
    for (int t = 0; t < PIX; ++t) {
        const int m0 = t * BM;
        const int s = pad_row(m0 + BM - 1) - pad_row(m0) + 2 * (PADW + 1) + 1;
        mx = s > mx ? s : mx;
    }
    return mx;
}

// per-channel vectors an operand prologue stages in LDS (PRO, below: 0 none; 1, 2 BN
// scale / shift)
constexpr int pro_params(int PRO) { return PRO != 0 ? 2 : 0; }

// LDS: halo rows [HR][32] + two weight chunks [2][BN][32] (register staging), or
// two halo buffers [2][HRG][32] + [2][BN][32] (LDS-DMA staging, VAR bit 4); the
// epilogue reuses it as a [BM][ELD] tile.
template <int C, int BN, int WM, int TM, int NW, int VAR = 0, int PRO = 0>
constexpr int halo_lds_bytes()
{
    using T = ConvTile<C, BN, WM, TM, NW>;
    const int hrg = (halo_span(T::BM) + 7) / 8 * 8;
    const int staging = (VAR & 4) ? (2 * hrg + ((VAR & 2) ? 3 : 2) * BN) * T::BK * 4
                                  : ((halo_span(T::BM) + T::RPP - 1) / T::RPP * T::RPP + 2 * BN) * T::BK * 4 +
                                        pro_params(PRO) * C * 4;
    const int epilogue = T::BM * (BN + 8) * 4;
    return staging > epilogue ? staging : epilogue;
}

// Tower epilogue: BN scale/shift, residual added when `resid` is non-null, ReLU
// (EPI_BN_RELU / EPI_BN_RES_RELU chosen at run time, same arithmetic).
constexpr int EPI_BN_OPTRES_RELU = 4;

// Train-step epilogue extras (template XE of halo_tile / halo_epilogue), computed
// from the tile while it is on chip so no separate pass re-reads the conv output:
//  XE_STATS  (train forward, EPI_RAW): per M tile and output channel the mean and
//            M2 = S (z - mean)^2 of the tile's valid rows (two-pass, fp32) ->
//            pa / pb [mtile][C]; the batch statistics combine the tiles exactly in
//            fp64 (bn_finalize_tiles_kernel, Chan's formula).
//  XE_BNBWD  (dgrad, EPI_RAW / EPI_ADD): the output g is the gradient of a BN+ReLU
//            output; per M tile and channel S dy and S (z - mean) dy with
//            dy = g * (act > 0) -> pa / pb [mtile][C] (BatchNorm backward sums).
constexpr int XE_NONE = 0;
constexpr int XE_STATS = 1;
constexpr int XE_BNBWD = 2;
struct EpiX {
    const float* act;    // XE_BNBWD: post-ReLU activation (mask)
    const float* z;      // XE_BNBWD: BN input
    const float* mean;   // XE_BNBWD: batch mean of z per channel
    float* pa;           // [mtiles][C]
    float* pb;           // [mtiles][C]
};


// BatchNorm finalize from per-tile partials (pa / pb [ntile][ldc]), shared by the
// stand-alone finalize kernels (pv_train.hip) and the last-arriving workgroup of a
// train conv (halo_epilogue, FinX): 8 consecutive lanes own one channel, lane j sums
// tiles j, j+8, ... in fp64, then a fixed xor tree over the 8 lanes -- the same
// order everywhere, so a fused and a separate finalize are bitwise identical.
//   FWD (train-forward statistics; pa = tile mean, pb = tile M2, tile t holds
//     min(prow, M - t*prow) rows): mean = S n_t m_t / N, var = (S (M2_t + n_t m_t^2)
//     - N mean^2) / N in fp64; invstd / scale / shift and the running-stat update as
//     ATen's CPU batch_norm (network.py:12-25 in train mode, momentum 0.1,
//     unbiased running var);
//   !FWD (BN backward; pa = S dy, pb = S (z - mean) dy): dgamma, dbeta and the
//     bn_bwd_apply coefficients gm = S dy / N, k = S(z-mean)dy invstd^2 / N,
//     iw = invstd * gamma.
struct FinX {
    unsigned* cnt = nullptr;     // fused: arrival counter per N tile (0 at launch; reset by the last arriver).
                                 // XE_STATS: the tile is stored after the arrival count, so the
                                 // write-through drain of the 32 KB tile leaves the finalize's path
    const float* gamma = nullptr;
    const float* beta = nullptr;                            // FWD
    float *rmean = nullptr, *rvar = nullptr;                // FWD running stats
    float *mean_o = nullptr, *inv_o = nullptr, *scale_o = nullptr, *shift_o = nullptr;   // FWD outputs
    const float* inv_i = nullptr;                           // !FWD: invstd of the layer
    float *ggamma = nullptr, *gbeta = nullptr;              // !FWD: parameter grads
    float *gm_o = nullptr, *k_o = nullptr, *iw_o = nullptr; // !FWD: bn_bwd_apply coefficients
};
// partial sums of tiles t = j, j+8, ... (the tile class j of 8) for channel c
template <bool FWD>
__device__ __forceinline__ void bn_fin_accum(const float* __restrict__ pa, const float* __restrict__ pb, int ldc,
                                             int ntile, int prow, int M, int c, int j, double& v0, double& v1)
{
    v0 = 0.0;
    v1 = 0.0;
    // loads of up to 32 tiles issued back to back before their sums (one round trip
    // per 32 tiles: unconditional loads from clamped rows, past-the-end tiles add an
    // exact 0 -- no branch between a load and the next)
    for (int t0 = j; t0 < ntile; t0 += 8 * 32) {
        float a[32], b[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const int t = min(t0 + 8 * k, ntile - 1);
            a[k] = pa[(size_t)t * ldc + c];
            b[k] = pb[(size_t)t * ldc + c];
        }
        __builtin_amdgcn_sched_barrier(0);   // hipcc otherwise interleaves each load with its wait
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const int t = t0 + 8 * k;
            const bool ok = t < ntile;
            if (FWD) {
                const double n = ok ? (double)min(prow, M - t * prow) : 0.0;
                const double av = (double)a[k];
                v0 += n * av;
                v1 += (ok ? (double)b[k] : 0.0) + n * av * av;
            } else {
                v0 += ok ? (double)a[k] : 0.0;
                v1 += ok ? (double)b[k] : 0.0;
            }
        }
    }
}
// combine the 8 tile classes in the fixed order ((0+4)+(2+6))+((1+5)+(3+7)) and write
// channel c's results
template <bool FWD>
__device__ __forceinline__ void bn_fin_out(double v0, double v1, int M, int c, const FinX& f)
{
    if (FWD) {
        const double mean = v0 / (double)M;
        double q = v1 - (double)M * mean * mean;     // S (z - mean)^2
        q = q > 0.0 ? q : 0.0;
        const double var = q / (double)M;
        const float mean_f = (float)mean;
        const float inv_f = (float)(1.0 / sqrt(var + (double)BN_EPS));
        const float alpha = inv_f * f.gamma[c];
        f.mean_o[c] = mean_f;
        f.inv_o[c] = inv_f;
        f.scale_o[c] = alpha;
        f.shift_o[c] = fmaf(-mean_f, alpha, f.beta[c]);
        const double unb = M > 1 ? q / (double)(M - 1) : var;
        f.rmean[c] = (float)((double)BN_MOMENTUM * mean + (1.0 - (double)BN_MOMENTUM) * (double)f.rmean[c]);
        f.rvar[c] = (float)((double)BN_MOMENTUM * unb + (1.0 - (double)BN_MOMENTUM) * (double)f.rvar[c]);
    } else {
        const double inv = (double)f.inv_i[c];
        f.ggamma[c] = (float)(v1 * inv);
        f.gbeta[c] = (float)v0;
        f.gm_o[c] = (float)(v0 / (double)M);
        f.k_o[c] = (float)(v1 * inv * inv / (double)M);
        f.iw_o[c] = (float)inv * f.gamma[c];
    }
}
// 8 waves x 64 lanes: wave w holds tile class w of channel c (lane); the classes are
// combined through LDS in the fixed order above by wave 0, which writes the results
// (shared by the fused finalize of halo_epilogue and the stand-alone kernels).
// Every thread of the workgroup must call it (barrier).  A 16-wave workgroup runs two
// such groups side by side (waves 8-15: the next 64 channels, `grp` 1): same order.
template <bool FWD>
__device__ __forceinline__ void bn_fin_combine8(double v0, double v1, double* red, int M, int c, bool valid,
                                                const FinX& f)
{
    const int wv = (threadIdx.x >> 6) & 7, ln = threadIdx.x & 63, grp = threadIdx.x >> 9;
    double* r0 = red + grp * 1024;
    r0[wv * 64 + ln] = v0;
    r0[512 + wv * 64 + ln] = v1;
    __syncthreads();
    if (wv == 0 && valid) {
        auto comb = [&](const double* r) {
            return ((r[0 * 64 + ln] + r[4 * 64 + ln]) + (r[2 * 64 + ln] + r[6 * 64 + ln])) +
                   ((r[1 * 64 + ln] + r[5 * 64 + ln]) + (r[3 * 64 + ln] + r[7 * 64 + ln]));
        };
        bn_fin_out<FWD>(comb(r0), comb(r0 + 512), M, c, f);
    }
}

// Train-forward operand prologue (template PRO of halo_tile): the conv input is the
// previous layer's RAW conv output z, and its BatchNorm (batch statistics) + ReLU
// (+ the block's residual input) is applied while the halo rows are staged:
//   a = relu(fma(z, scale[c], shift[c]) [+ res])   (padding rows stay 0)
// so no separate bn_apply pass reads z and writes a; the tile's own pixel rows of
// a (needed by the backward) are written once, by the N-tile-0 workgroups.
constexpr int PRO_NONE = 0;
constexpr int PRO_BN = 1;       // relu(bn(z))
constexpr int PRO_BN_RES = 2;   // relu(bn(z) + res)
#ifndef AZG_PRO_REMAT
#define AZG_PRO_REMAT 1
#endif
struct ProX {
    const float* res;     // PRO_BN_RES: residual input
    const float* scale;   // [C] BN scale of the input layer (invstd * gamma)
    const float* shift;   // [C] beta - mean * scale
    float* aout;          // a (padded NHWC): own rows written when n0 == 0
};


// H3 range guard: an activation at or above 65520 rounds to an infinite hi part, and
// every product it enters becomes inf - inf or 0 * inf = NaN, so a non-finite
// accumulator in the epilogue means an input left fp16's range: the tile posts its
// launch number to the handle's host ring (the host recomputes that forward with fp32
// MFMA, azg_pv_recover) and computes on.  (Below 65520 the split is exact as usual.)
struct H3Guard {
    unsigned* ring = nullptr;   // host-mapped, kTowerRing entries (device alias)
    unsigned seq = 0;
    // split-fp16 dgrad (XE_BNBWD): the bits of max |input| of the layer (bn_bwd_apply's
    // atomicMax); the input is staged times 2^k so its largest element lies in [2^14, 2^15)
    // (fp16's top binade: every element keeps a normal hi part down to 2^-28 of the max),
    // and the epilogue's factor carries 2^-k
    const unsigned* dmax = nullptr;
};
// k of the dgrad input scale 2^k for max |input| bits `maxbits` (0: an all-zero input)
__device__ __forceinline__ int h3_dgrad_exp(unsigned maxbits)
{
    const float m = __uint_as_float(maxbits);
    const int k = m > 0.f && __builtin_isfinite(m) ? 14 - ilogbf(m) : 0;
    return k < -100 ? -100 : k > 100 ? 100 : k;   // 2^k and the epilogue's 2^-(e + k) stay normal
}
constexpr unsigned kH3RingSize = 256;   // = kTowerRing (pv_internal.h)

// key of the 16-B slot swizzle of halo row `row` (padded-pixel index): the padded
// board position v = yy*15 + xx (see halo_tile)
__device__ __forceinline__ int halo_vkey(int row)
{
    const int rb = row % PADPIX;
    return (rb / PADW) * BOARD + rb % PADW;
}

// Epilogue through LDS: the accumulators (C/D map of the 32x32 MFMA: col =
// lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)) are written to an LDS tile
// [BM][ELD] (ELD = BN: the ds_write_b32 halves and the ds_read_b128 lane groups
// are conflict-free on unpadded rows; BN+8 conflicts on the reads), then every
// thread finishes 16-B runs of 4 channels of one pixel: one pad_off, float4
// scale/shift/residual, one 16-B store per run -- instead of 16 scalar stores (and
// 16 pad_off divisions) per fragment.  Same per-element arithmetic.  The caller
// guarantees every wave is past its last staging-buffer access (barrier).
// RBUF: how the residual is read -- 0 plain pointer loads; 1 buffer loads (default
// cache policy); 2 buffer loads with sc1 (the tower's one-workgroup-per-CU hand-off)
template <int C, int BN_, int WM_, int TM_, int NW_, int EPI, bool SC1, int ABL, int ELD, bool EARLY = false,
          int XE = XE_NONE, int RBUF = 0>
__device__ __forceinline__ void halo_epilogue(const f32x16 (&acc)[TM_][ConvTile<C, BN_, WM_, TM_, NW_>::TN],
                                              const float* __restrict__ scale, const float* __restrict__ shift,
                                              const float* __restrict__ resid, float* __restrict__ out,
                                              __amdgpu_buffer_rsrc_t out_rs, int M, int m0, int n0, float* smem,
                                              const EpiX& ex = EpiX{}, const FinX& fx = FinX{},
                                              const H3Guard* guard = nullptr)
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    constexpr int BM = T::BM, BN = T::BN, WN = T::WN, TM = T::TM, TN = T::TN;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int r32 = lane & 31, h = lane >> 5;
    float* Es = smem;
    constexpr int CPR = BN / 4;            // 16-B runs per pixel row
    constexpr int RPI = T::NT / CPR;       // pixel rows per pass
    constexpr int NPASS = BM / RPI;
    static_assert(BM % RPI == 0, "epilogue passes");
    const int ec = (tid % CPR) * 4;
    const int er = tid / CPR;
    const int col = n0 + ec;
    const bool has_res = EPI == EPI_BN_RES_RELU || EPI == EPI_ADD || (EPI == EPI_BN_OPTRES_RELU && resid);
    // EARLY: the residual / scale / shift loads are issued before the accumulator
    // tile goes through LDS, so their latency overlaps the ds_write + barrier
    f32x4 rve[EARLY ? NPASS : 1];
    f32x4 s4 = {1.f, 1.f, 1.f, 1.f}, t4 = {0.f, 0.f, 0.f, 0.f};
    if (EARLY) {
        if (EPI == EPI_BN_RELU || EPI == EPI_BN_RES_RELU || EPI == EPI_BN_OPTRES_RELU) {
            s4 = *(const f32x4*)(scale + col);
            t4 = *(const f32x4*)(shift + col);
        }
#pragma unroll
        for (int p = 0; p < (EARLY ? NPASS : 1); ++p) {
            const int m = m0 + er + p * RPI;
            rve[p] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (has_res && m < M) rve[p] = *(const f32x4*)(resid + pad_off(m, C) + col);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                Es[row * ELD + wn * TN * 32 + j * 32 + r32] = acc[i][j][r];
            }
    __syncthreads();
    f32x4 h3s = {1.f, 1.f, 1.f, 1.f};
    if ((EPI == EPI_RAW || EPI == EPI_ADD) && guard) {
        h3s = *(const f32x4*)(scale + col);
        if (guard->dmax) h3s *= ldexpf(1.f, -h3_dgrad_exp(*guard->dmax));   // the dgrad input's 2^-k: exact
    }
    if (!EARLY && (EPI == EPI_BN_RELU || EPI == EPI_BN_RES_RELU || EPI == EPI_BN_OPTRES_RELU)) {
        s4 = *(const f32x4*)(scale + col);
        t4 = *(const f32x4*)(shift + col);
    }
    // XE partials of this thread's 4 channels over its rows
    f32x4 xa = {0.f, 0.f, 0.f, 0.f}, xb = {0.f, 0.f, 0.f, 0.f}, xmu = {0.f, 0.f, 0.f, 0.f};
    f32x4 vk[XE == XE_STATS ? NPASS : 1];
    // late store (XE_STATS + fused finalize): the raw tile (kept in vk) is stored after the
    // partials are published and counted, so the arrival waits only for the partials
    const bool late = XE == XE_STATS && EPI == EPI_RAW && fx.cnt != nullptr;
    if (XE == XE_BNBWD) xmu = *(const f32x4*)(ex.mean + col);
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
        const int row = er + p * RPI;
        const int m = m0 + row;
        f32x4 v = *(const f32x4*)(Es + row * ELD + ec);
        if ((EPI == EPI_RAW || EPI == EPI_ADD) && guard) v *= h3s;   // split-fp16 weights carry 2^e: exact
        if (guard) {   // H3: a non-finite accumulator = an input beyond fp16's range (H3Guard)
            const bool fin = __builtin_isfinite(v[0]) && __builtin_isfinite(v[1]) && __builtin_isfinite(v[2]) &&
                             __builtin_isfinite(v[3]);
            if (!fin && m0 + row < M && guard->ring && guard->seq)
                __hip_atomic_store(guard->ring + (guard->seq & (kH3RingSize - 1)), guard->seq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (XE == XE_STATS) vk[p] = v;
        if (m < M && (!(ABL & 16) || v[0] == 1234.5f)) {
            const int o = pad_off(m, C) + col;
            f32x4 xact, xz;
            if (XE == XE_BNBWD) {
                xact = *(const f32x4*)(ex.act + o);
                xz = *(const f32x4*)(ex.z + o);
            }
            f32x4 rv = {0.f, 0.f, 0.f, 0.f};
            if (EARLY) rv = rve[EARLY ? p : 0];
            else if (has_res && RBUF)   // residual produced inside the launch (tower)
                rv = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(resid), (short)0,
                                                                                     0x7fffffff, 0x00020000),
                                                   o * 4, 0, RBUF == 2 ? 16 : 0));
            else if (has_res) rv = *(const f32x4*)(resid + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = v[e];
                // explicit fmaf: the same rounding in every epilogue form (a contracted
                // x * s + t in one kernel and an uncontracted one in another made the
                // tower and the per-layer launches differ by an ulp once BN shifts are
                // nonzero -- trained nets; seeded ones have shift 0)
                if (EPI == EPI_BN_RELU) {
                    x = fmaxf(fmaf(x, s4[e], t4[e]), 0.f);
                } else if (EPI == EPI_BN_RES_RELU) {
                    x = fmaxf(fmaf(x, s4[e], t4[e]) + rv[e], 0.f);
                } else if (EPI == EPI_BN_OPTRES_RELU) {
                    x = has_res ? fmaxf(fmaf(x, s4[e], t4[e]) + rv[e], 0.f) : fmaxf(fmaf(x, s4[e], t4[e]), 0.f);
                } else if (EPI == EPI_ADD) {
                    x = x + rv[e];
                }
                v[e] = x;
            }
            if (XE == XE_STATS) xa += v;
            if (XE == XE_BNBWD) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float dy = xact[e] > 0.f ? v[e] : 0.f;
                    xa[e] += dy;
                    xb[e] = fmaf(xz[e] - xmu[e], dy, xb[e]);
                }
            }
            if (!late) {
                if constexpr (SC1) {
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), out_rs, o * 4, 0, 16);
                } else {
                    *(f32x4*)(out + o) = v;
                }
            }
        }
    }
    if constexpr (XE != XE_NONE) {
        // fixed-order LDS reduction over the RPI row groups (bitwise reproducible)
        static_assert(2 * RPI * BN + BN + 1 <= BM * ELD, "XE reduction scratch (+ arrival flag)");
        float* R = smem;                       // [RPI][BN] partial a, then [RPI][BN] partial b
        float* Mu = smem + 2 * RPI * BN;       // [BN] tile mean (XE_STATS)
        const int mt = m0 / BM;
        const int ntm = (M + BM - 1) / BM;
        const int rows = min(BM, M - m0);
        // partials are stored write-through: a fused finalize (fx.cnt) reads them from
        // another XCD after the arrival count
        const __amdgpu_buffer_rsrc_t prs_a = wt_rsrc(ex.pa, (size_t)ntm * C * sizeof(float));
        const __amdgpu_buffer_rsrc_t prs_b = wt_rsrc(ex.pb, (size_t)ntm * C * sizeof(float));
        const int po = mt * C + n0 + tid;
        __syncthreads();                       // every thread is past its Es reads
        *(f32x4*)(R + er * BN + ec) = xa;
        if (XE == XE_BNBWD) *(f32x4*)(R + RPI * BN + er * BN + ec) = xb;
        __syncthreads();
        if (tid < BN) {
            float sa = 0.f, sb = 0.f;
            for (int r = 0; r < RPI; ++r) sa += R[r * BN + tid];
            if (XE == XE_BNBWD) {
                for (int r = 0; r < RPI; ++r) sb += R[RPI * BN + r * BN + tid];
                store1<true>(ex.pa, prs_a, po, sa);
                store1<true>(ex.pb, prs_b, po, sb);
            } else {
                const float mu = sa / (float)rows;
                Mu[tid] = mu;
                store1<true>(ex.pa, prs_a, po, mu);
            }
        }
        if constexpr (XE == XE_STATS) {
            __syncthreads();
            const f32x4 mu4 = *(const f32x4*)(Mu + ec);
            f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int p = 0; p < NPASS; ++p) {
                if (er + p * RPI < rows) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = vk[p][e] - mu4[e];
                        q[e] = fmaf(d, d, q[e]);
                    }
                }
            }
            *(f32x4*)(R + RPI * BN + er * BN + ec) = q;
            __syncthreads();
            if (tid < BN) {
                float sb = 0.f;
                for (int r = 0; r < RPI; ++r) sb += R[RPI * BN + r * BN + tid];
                store1<true>(ex.pb, prs_b, po, sb);
            }
        }
        // fused finalize: the last workgroup of this N tile to publish its partials
        // reduces all M tiles' partials of its BN channels.  Hand-off (MI355X_MICROARCH
        // "Valid forms", producer R1 + consumer acquire -- the form valid at any number
        // of workgroups per CU; this launch runs two): write-through stores, every wave
        // vmcnt(0), barrier, one agent-scope atomic add per workgroup; the workgroup
        // whose add returns ntm - 1 runs ONE agent-scope acquire, vmcnt(0) and a barrier
        // before its plain loads of the partials.
        if (fx.cnt) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            unsigned* flag = (unsigned*)(smem + 2 * RPI * BN + BN);
            if (tid == 0) {
                const unsigned old =
                    __hip_atomic_fetch_add(fx.cnt + n0 / BN, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned last = old == (unsigned)(ntm - 1) ? 1u : 0u;
                if (last) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                *flag = last;
            }
            __syncthreads();
            if constexpr (XE == XE_STATS) {
                if (late) {   // the tile (= vk, EPI_RAW) now; it drains while the finalize runs
#pragma unroll
                    for (int p = 0; p < NPASS; ++p) {
                        const int m = m0 + er + p * RPI;
                        if (m < M) {
                            const int o = pad_off(m, C) + col;
                            if constexpr (SC1) {
                                __builtin_amdgcn_raw_buffer_store_b128(
                                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vk[p]), out_rs,
                                    o * 4, 0, 16);
                            } else {
                                *(f32x4*)(out + o) = vk[p];
                            }
                        }
                    }
                }
            }
            if (*flag) {
                // wave w sums tile class w % 8 of channels n0 + lane (coalesced rows of
                // the [tile][C] partials), the classes combine through LDS in the order
                // of bn_fin_combine8: bitwise equal to the stand-alone finalize
                // (16 waves x 128 channels: waves 8-15 do channels n0 + 64 + lane)
                static_assert((T::NW == 8 && BN == 64) || (T::NW == 16 && BN == 128),
                              "fused finalize: 8 waves per 64 channels");
                static_assert(2 * 1024 * 8 <= BM * ELD * 4, "fused finalize: LDS for the combine");
                double* red = (double*)smem;   // [groups][2][8][64]
                const int wv = (tid >> 6) & 7, ln = tid & 63, ch = n0 + (tid >> 9) * 64 + ln;
                double v0, v1;
                bn_fin_accum<XE == XE_STATS>(ex.pa, ex.pb, C, ntm, BM, M, ch, wv, v0, v1);
                bn_fin_combine8<XE == XE_STATS>(v0, v1, red, M, ch, true, fx);
                if (tid == 0) __hip_atomic_store(fx.cnt + n0 / BN, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Main loop with LDS-DMA staging (VAR bit 4): every operand reaches LDS through
// global_load_lds_dwordx4 (one wave-instruction = 1 KiB = 8 rows of 128 B, written
// lane-linearly; the slot swizzle is applied to each lane's SOURCE address, and the
// fragment reads use the same swizzle -- cdna_hip_programming.md §5.4 rule 21), so
// no VGPR holds staged data and no ds_write is issued.  The halo is double-buffered
// (group g+1's pieces are issued over the first taps of group g), so the extra
// per-group barrier of the register path disappears; weights of chunk j+1 are issued
// at the top of chunk j.  Ordering: every chunk ends with __syncthreads (its fence
// waits vmcnt(0), retiring that chunk's DMAs before the barrier), data is read one
// chunk after the barrier that retired it, and a buffer is refilled one chunk after
// the barrier that ended its last read.  Same K order and chains as halo_tile.
template <int C, int BN_, int WM_, int TM_, int NW_, int VAR>
__device__ __forceinline__ void halo_mainloop_glds(const float* __restrict__ in, const float* __restrict__ wp,
                                                   int M, int m0, int n0, float* smem,
                                                   f32x16 (&acc)[TM_][ConvTile<C, BN_, WM_, TM_, NW_>::TN])
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    constexpr int BM = T::BM, BN = T::BN, BK = T::BK;
    constexpr int CG = T::CG, WN = T::WN, TM = T::TM, TN = T::TN, NW = T::NW;
    constexpr int HS = halo_span(BM);
    constexpr int NP = (HS + 7) / 8;          // halo pieces (8 rows each)
    constexpr int HRG = NP * 8;
    constexpr int NPW = (NP + NW - 1) / NW;   // halo pieces per wave
    constexpr int NBP = BN / 8;               // weight pieces per chunk
    constexpr int NBW = (NBP + NW - 1) / NW;
    constexpr int NCHK = 9 * CG;
    constexpr bool VSWZ = (VAR & 1) != 0;
    // PF2 (VAR bit 2): three weight buffers, chunk j+2 issued at the top of chunk j and
    // kept in flight across the chunk-end barrier (raw s_barrier + counted vmcnt
    // instead of __syncthreads, whose fence drains every DMA)
    constexpr bool PF2 = (VAR & 2) != 0;
    constexpr int NWB = PF2 ? 3 : 2;
    constexpr int NPF = NP / NW;              // taps at which EVERY wave issues a halo piece
    static_assert(!PF2 || NBP % NW == 0, "counted waits need the same weight pieces per wave");
    static_assert(NPW <= 9, "halo pieces are spread over the 9 taps");
    static_assert(BN % 8 == 0, "weight pieces");

    float* Ah = smem;                  // [2][HRG][32]
    float* Bs = smem + 2 * HRG * BK;   // [2][BN][32]
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int mlast = min(m0 + BM, M) - 1;
    const int hbase = pad_row(m0) - (PADW + 1);
    const int hmax = pad_row(mlast) + (PADW + 1);
    const int lr = lane >> 3, ls = lane & 7;   // row in piece, LDS slot of this lane

    int hoff[NPW];
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
        const int l = 8 * (wid + NW * i) + lr;            // LDS halo row
        const int key = VSWZ ? (halo_vkey(hbase + l) >> 1) & 7 : (l >> 1) & 7;
        hoff[i] = min(hbase + l, hmax) * C + ((ls ^ key) * 4);
    }
    int woff[NBW];
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
        const int n = 8 * (wid + NW * i) + lr;
        woff[i] = (n0 + n) * BK + ((ls ^ ((n >> 1) & 7)) * 4);
    }
    auto glds = [](const float* src, float* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    auto hpiece = [&](int g, int i) {
        const int p = wid + NW * i;
        if (p < NP) glds(in + g * BK + hoff[i], Ah + (g & 1) * HRG * BK + p * 8 * BK);
    };
    auto bchunk = [&](int j) {
        const float* wk = wp + (size_t)((j % 9) * CG + j / 9) * C * BK;
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
            const int p = wid + NW * i;
            if (p < NBP) glds(wk + woff[i], Bs + (j % NWB) * BN * BK + p * 8 * BK);
        }
    };

    const int r32 = lane & 31, h = lane >> 5;
    int hrow[TM], vpix[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int pr = pad_row(min(m0 + wm * TM * 32 + i * 32 + r32, M - 1));
        hrow[i] = pr - hbase;
        vpix[i] = halo_vkey(pr);
    }
    const int bswz = (r32 >> 1) & 7;
    const int brow = (wn * TN * 32 + r32) * BK;

#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // vmcnt(n) with n an unrolled-loop constant
    auto wait_vm = [](int n) {
        if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
    };
    // halo pieces every wave issued at chunk k (the smaller count where waves differ:
    // a conservative wait, never a short one)
    auto hcount = [&](int k) { return (k >= 0 && k / 9 + 1 < CG && k % 9 < NPF) ? 1 : 0; };

#pragma unroll
    for (int i = 0; i < NPW; ++i) hpiece(0, i);
    bchunk(0);
    if (PF2) {
        bchunk(1);
        wait_vm(NBW);            // halo of group 0 and weights of chunk 0 have landed
        raw_barrier();
    } else {
        __syncthreads();
    }

#pragma unroll
    for (int cg = 0; cg < CG; ++cg) {
        f32x16 at[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) at[i][j][r] = 0.f;
        const float* Ab = Ah + (cg & 1) * HRG * BK;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int j = cg * 9 + tap;
            if (PF2) {
                if (j + 2 < NCHK) bchunk(j + 2);
            } else {
                if (j + 1 < NCHK) bchunk(j + 1);
            }
            if (cg + 1 < CG && tap < NPW) hpiece(cg + 1, tap);
            __builtin_amdgcn_sched_barrier(0);
            const int d = (tap / 3 - 1) * PADW + (tap % 3 - 1);
            const int vd = (tap / 3 - 1) * BOARD + (tap % 3 - 1);
            int arow[TM], aswz[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = hrow[i] + d;
                arow[i] = r * BK;
                aswz[i] = VSWZ ? ((vpix[i] + vd) >> 1) & 7 : (r >> 1) & 7;
            }
            const float* Bb = Bs + (j % NWB) * BN * BK;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 a[TM], b[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) a[i] = *(const f32x4*)(Ab + arow[i] + (((h * 4 + q) ^ aswz[i]) * 4));
                const int rc = ((h * 4 + q) ^ bswz) * 4;
#pragma unroll
                for (int jn = 0; jn < TN; ++jn) b[jn] = *(const f32x4*)(Bb + brow + jn * 32 * BK + rc);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int jn = 0; jn < TN; ++jn)
                            at[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[jn][s], at[i][jn], 0, 0, 0);
            }
            if (PF2) {
                // retire weights(j+1) (and, in order, everything issued before it: the
                // next group's halo pieces); what was issued after it may stay in flight
                wait_vm(hcount(j - 1) + (j + 2 < NCHK ? NBW : 0) + hcount(j));
                raw_barrier();
            } else {
                __syncthreads();
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] += at[i][j];
    }
}

// One BM x BN output tile at (m0, n0).  K is ordered input-channel-group major:
// for each 32-wide channel group cg the tile's halo slice [rows][32] is staged into
// LDS ONCE and all 9 taps read their shifted A fragments from it (9x fewer A loads
// from L2 than staging an A tile per (tap, cg) chunk); the weights stream per chunk
// through a double-buffered LDS tile.  Accumulation: one MFMA chain per channel
// group over its 9 taps x 32 channels (288 terms), group sums added in cg order --
// error growth chain(288) + C/32, cf. chain(9C) for a single chain.  The K order
// is per output element and the same for every tile shape and position, so tuning
// never changes numerics and the forward is batch-independent.  Halo rows are
// staged through registers (loads issued over the first taps of the previous
// group) into a single LDS buffer, swapped behind one extra barrier per group.
//
// SC1: outputs are stored write-through (buffer_store ... sc1 via `out_rs`) so a
// consumer workgroup of the same launch can read them after its acquire
// (cdna_hip_programming.md Guideline 16, R1).
//
// ABL (timing studies only, 0 in every product launch; results are garbage when
// set): bit 1 skips the weight loads, bit 2 the halo loads, bit 4 the per-chunk
// barriers, bit 8 replaces LDS fragment reads by register values, bit 16 skips the
// epilogue stores (kept live by a never-true compare).
template <int C, int BN_, int WM_, int TM_, int NW_, int EPI, bool SC1 = false, int ABL = 0, int VAR = 0,
          int XE = XE_NONE, int PRO = PRO_NONE>
__device__ __forceinline__ void halo_tile(
    const float* __restrict__ in, const float* __restrict__ wp,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ resid, float* __restrict__ out, __amdgpu_buffer_rsrc_t out_rs,
    int M, int m0, int n0, float* smem, const EpiX& ex = EpiX{}, const ProX& px = ProX{},
    const FinX& fx = FinX{}, const H3Guard& guard = H3Guard{})
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    if constexpr ((VAR & 4) != 0) {   // LDS-DMA staging
        f32x16 acc[TM_][T::TN];
        halo_mainloop_glds<C, BN_, WM_, TM_, NW_, VAR>(in, wp, M, m0, n0, smem, acc);
        halo_epilogue<C, BN_, WM_, TM_, NW_, EPI, SC1, ABL, T::BN, (VAR & 8) != 0>(acc, scale, shift, resid, out,
                                                                                   out_rs, M, m0, n0, smem);
        return;
    }
    constexpr int RPP = T::RPP;
    constexpr int BM = T::BM, BN = T::BN, BK = T::BK;
    constexpr int CG = T::CG, WN = T::WN, TM = T::TM, TN = T::TN;
    constexpr int B_LD = T::B_LD;
    constexpr int HS = halo_span(BM);
    constexpr int H_LD = (HS + RPP - 1) / RPP;
    constexpr int HR = H_LD * RPP;
    static_assert(RPP % 16 == 0, "halo staging rows must keep the row swizzle");
    static_assert(H_LD <= 9, "halo loads are spread over the 9 taps");
    static_assert(PRO == PRO_NONE || H_LD <= 8, "the operand prologue of a row runs one tap after its load");
    static_assert(PRO == PRO_NONE || (((VAR & ~193) == 0 || (VAR & ~193) == 32) && ABL == 0),
                  "operand prologue: register staging only");
    // VAR (A/B studies; the product uses 0, measured fastest): bit 1 = halo rows
    // swizzled on the padded board position (conflict-free fragment reads) and an
    // unpadded epilogue tile; bit 2 = weights staged two chunks ahead; bit 4 = LDS-DMA
    // staging (halo_mainloop_glds); bit 8 = epilogue loads issued before the LDS pass.  Every VAR computes bitwise-identical results.
    constexpr bool VSWZ = (VAR & 1) != 0;
    constexpr bool BPF2 = (VAR & 2) != 0;
    // H3 (VAR bit 64, eval only): fp32-equivalent products from three fp16 MFMAs.  Every
    // operand x is split into hi = fp16(x) and lo = fp16(x - hi) (x = hi + lo to 2^-22 of
    // x, or 3e-8 absolute below fp16's normal range); a K16 step is acc += lo_a hi_b +
    // hi_a lo_b + hi_a hi_b (v_mfma_f32_32x32x16_f16: exact 22-bit products, fp32
    // accumulation), the dropped lo_a lo_b is 2^-22 of the product.  A 128-B LDS row of 32
    // channels holds [hi 32 x fp16 | lo 32 x fp16]: the fp32 row geometry, so the 16-B slot
    // swizzles are unchanged.  Halo rows are split while staged; weights are packed split
    // (and scaled by a per-layer power of two so their lo parts stay normal,
    // pv_pack.hip pack_h3; the epilogue's BN scale carries the inverse).
    constexpr bool H3 = (VAR & 64) != 0;
    // train forward (EPI_RAW + XE_STATS, PRO): BN-normalised inputs; the raw output is
    // multiplied by `scale` (2^-e of the layer) in the epilogue.  Dgrad (EPI_RAW / EPI_ADD +
    // XE_BNBWD, key 50): the input gradient is not normalised -- it is staged times 2^k from
    // its measured max (H3Guard::dmax) and the epilogue's factor is 2^-(e + k), applied
    // before the residual gradient is added.
    static_assert(!H3 || XE == XE_NONE || XE == XE_STATS || (XE == XE_BNBWD && PRO == PRO_NONE),
                  "H3: eval, train-forward and dgrad tiles");
    const float dsc = (H3 && XE == XE_BNBWD && guard.dmax) ? ldexpf(1.f, h3_dgrad_exp(*guard.dmax)) : 1.f;
    constexpr int NCHK = 9 * CG;

    float* Ah = smem;                 // [HR][32]
    float* Bs = smem + HR * BK;       // [2][BN][32]
    float* Ps = smem + (HR + 2 * BN) * BK;   // PRO: [2][C] input-layer BN scale / shift

    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int mlast = min(m0 + BM, M) - 1;
    const int hbase = pad_row(m0) - (PADW + 1);
    const int hmax = pad_row(mlast) + (PADW + 1);

    const int sr = tid >> 3, sc = (tid & 7) * 4;
    int hsrc[H_LD];
#pragma unroll
    for (int i = 0; i < H_LD; ++i) {
        const int r = min(hbase + sr + RPP * i, hmax);   // rows past the tile's need: any valid row
        hsrc[i] = r * C + sc;
    }
    const float* wsrc = wp + (size_t)(n0 + sr) * BK + sc;
    // PRO: per staged row, interior (else the zero halo) / own pixel row (write a)
    unsigned pint = 0, pown = 0;   // own rows are never clamped: their a offset is hsrc[i]
    if constexpr (PRO != PRO_NONE) {
        const int own_lo = pad_row(m0), own_hi = pad_row(mlast);
#pragma unroll
        for (int i = 0; i < H_LD; ++i) {
            const int r = hbase + sr + RPP * i;
            const int rb = r % PADPIX, yy = rb / PADW, xx = rb - yy * PADW;
            const bool interior = yy >= 1 && yy <= BOARD && xx >= 1 && xx <= BOARD;
            if (interior) pint |= 1u << i;
            if (interior && n0 == 0 && r >= own_lo && r <= own_hi) pown |= 1u << i;
        }
        for (int c = tid; c < C; c += T::NT) {
            Ps[c] = px.scale[c];
            Ps[C + c] = px.shift[c];
        }
        __syncthreads();
    }

    // weights: rb1 holds chunk j+1 (stored to LDS at the end of chunk j); with BPF2,
    // rb2 receives chunk j+2 at the top of chunk j, so a load has a whole chunk plus
    // the next chunk's MFMAs to land before the ds_write that waits on it (the loops
    // are fully unrolled: the rb1 = rb2 hand-over is a register renaming, not a move)
    f32x4 rh[H_LD], rb1[B_LD], rb2[B_LD];
    f32x4 rr[PRO == PRO_BN_RES ? H_LD : 1];
    // VAR bit 16 (persistent tower at ONE workgroup per CU): halo rows are produced
    // inside the launch by other CUs; every load of them is an sc1 buffer load (L1
    // bypassed) in place of the consumer's acquire -- row 1 of the microarch guide's
    // measured hand-off table, valid only at one workgroup per CU (pv_tower.hip).
    // VAR bit 32: the same buffer-resource addressing (32-bit offsets: fewer VGPRs than
    // 64-bit pointers) with the default cache policy, behind the consumer's acquire.
    const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), (short)0,
                                                                          0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t res_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(px.res), (short)0,
                                                                           0x7fffffff, 0x00020000);
    // 1024-thread tiles stage 2 x 128 rows for a halo of at most HS rows: rows past the
    // tile's last needed row (hmax) are not loaded (their LDS rows are never read)
    constexpr bool HPRED = T::NT >= 1024 && H_LD * RPP - HS >= RPP / 4;
    if constexpr (HPRED) {
#pragma unroll
        for (int i = 0; i < H_LD; ++i) rh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto hload = [&](int cg, int i) {
        if (ABL & 2) return;
        if constexpr (HPRED) {
            if (hbase + sr + RPP * i > hmax) return;
        }
        if constexpr ((VAR & 48) != 0)
            rh[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, (hsrc[i] + cg * BK) * 4, 0,
                                                                                    (VAR & 16) ? 16 : 0));
        else
            rh[i] = *(const f32x4*)(in + hsrc[i] + cg * BK);
        if constexpr (PRO == PRO_BN_RES) {
            if constexpr ((VAR & 32) != 0)
                rr[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(res_rs, (hsrc[i] + cg * BK) * 4, 0, 0));
            else
                rr[i] = *(const f32x4*)(px.res + hsrc[i] + cg * BK);
        }
    };
    // VAR 16 / 32: weights through a buffer resource too (SGPR base + one VGPR offset
    // + per-chunk SGPR/immediate offsets, instead of a 64-bit address per chunk)
    const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wp), (short)0,
                                                                         0x7fffffff, 0x00020000);
    const int wvo = ((n0 + sr) * BK + sc) * 4;
    auto bload = [&](f32x4 (&rb)[B_LD], int kc) {
        if (ABL & 1) return;
        if constexpr ((VAR & 48) != 0) {
#pragma unroll
            for (int i = 0; i < B_LD; ++i)
                rb[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      w_rs, wvo, (kc * C * BK + RPP * i * BK) * 4, 0));
        } else {
            const float* wk = wsrc + (size_t)kc * C * BK;
#pragma unroll
            for (int i = 0; i < B_LD; ++i) rb[i] = *(const f32x4*)(wk + RPP * i * BK);
        }
    };
    // K chunk j (0 .. 9*CG-1) = tap j%9 of channel group j/9 -> packed weight chunk
    auto kchunk = [](int j) { return (j % 9) * CG + j / 9; };
    // LDS swizzles.  ds_read_b128 serves a wave in 4 lane groups of 16 (e.g. lanes
    // {0-3, 12-15, 20-27}); a group is conflict-free iff its 16 reads hit distinct
    // (row parity, 16-B slot) pairs.  Weight rows: chunk c of row r sits at slot
    // c ^ ((r >> 1) & 7) -- consecutive rows, conflict-free.  Halo rows: a fragment's
    // 32 lanes read the rows of 32 consecutive pixels, which jump by 3 padded rows at
    // each board-row end, so a row-keyed slot conflicts there (113 M conflict cycles
    // per tower launch, PMC).  VSWZ keys halo rows on v = yy*15 + xx of the padded
    // position (yy, xx): for every tap, consecutive pixels read consecutive v (across
    // row ends too) and the row parity alternates with v (row steps are 1 or 3), so
    // slot c ^ ((v >> 1) & 7) is conflict-free for every lane group inside a board.
    const int wchunk = ((tid & 7) ^ ((sr >> 1) & 7)) * 4;
    auto vkey = [](int row) { return halo_vkey(row); };
    int hwchunk[H_LD];
#pragma unroll
    for (int i = 0; i < H_LD; ++i)
        hwchunk[i] = VSWZ ? ((tid & 7) ^ ((vkey(hbase + sr + RPP * i) >> 1) & 7)) * 4 : wchunk;
    // PRO: the BN / residual / ReLU of the input layer on the staged rows (same
    // arithmetic as bn_apply_kernel), own rows of a written through
    const __amdgpu_buffer_rsrc_t ars = wt_rsrc(px.aout, padded_bytes(M, C));
    // per staged row i: applied one tap after its load was issued (the residual row
    // dies there, keeping the PRO_BN_RES register peak low), to all rows of the first
    // group before its store
    auto pro_row = [&](int cg, int i) {
        if constexpr (PRO != PRO_NONE) {
            const f32x4 s4 = *(const f32x4*)(Ps + cg * BK + sc);
            const f32x4 t4 = *(const f32x4*)(Ps + C + cg * BK + sc);
            f32x4 v = rh[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float y = fmaf(v[e], s4[e], t4[e]);
                if constexpr (PRO == PRO_BN_RES) y += rr[i][e];
                v[e] = (pint >> i) & 1 ? fmaxf(y, 0.f) : 0.f;
            }
            rh[i] = v;
            if ((pown >> i) & 1) store4<true>(px.aout, ars, hsrc[i] + cg * BK, v);
        }
    };
    auto hstore = [&](int cg) {
        if constexpr (H3) {
            // channels sc..sc+3 of the row: hi halves into slot sc/8 (byte 2*(sc%8)),
            // lo halves into slot 4 + sc/8, both slots swizzled like the fp32 row's
#pragma unroll
            for (int i = 0; i < H_LD; ++i) {
                const int key = (hwchunk[i] >> 2) ^ (tid & 7);   // the row's slot swizzle
                f16x4 hi, lo;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = XE == XE_BNBWD ? rh[i][e] * dsc : rh[i][e];   // dgrad: times 2^k (exact)
                    hi[e] = (_Float16)x;
                    lo[e] = (_Float16)(x - (float)hi[e]);
                }
                float* row = Ah + (sr + RPP * i) * BK;
                const int q = (tid & 7) >> 1, half = ((tid & 7) & 1) * 2;
                *(f16x4*)(row + ((q ^ key) * 4) + half) = hi;
                *(f16x4*)(row + (((4 + q) ^ key) * 4) + half) = lo;
            }
        } else {
#pragma unroll
            for (int i = 0; i < H_LD; ++i) *(f32x4*)(Ah + (sr + RPP * i) * BK + hwchunk[i]) = rh[i];
        }
    };
    auto bstore = [&](const f32x4 (&rb)[B_LD], int buf) {
        float* b = Bs + buf * BN * BK;
#pragma unroll
        for (int i = 0; i < B_LD; ++i) *(f32x4*)(b + (sr + RPP * i) * BK + wchunk) = rb[i];
    };

    // Lane l of an MFMA step s uses K index h*16+s (h = l>>5) for both A and B, so
    // each lane's 16 A values and 16 B values of a chunk are contiguous in LDS.
    const int r32 = lane & 31, h = lane >> 5;
    // halo row of each fragment pixel (tail pixels clamp to the last valid one)
    int hrow[TM], vpix[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int pr = pad_row(min(m0 + wm * TM * 32 + i * 32 + r32, M - 1));
        hrow[i] = pr - hbase;
        vpix[i] = vkey(pr);
    }
    const int bswz = (r32 >> 1) & 7;
    const int brow = (wn * TN * 32 + r32) * BK;
    const f32x4 rfix = {(float)r32, (float)h, 1.f, 2.f};   // ABL & 8 operands (timing only)

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
    for (int i = 0; i < H_LD; ++i) hload(0, i);
    if (BPF2) {
        bload(rb2, kchunk(0));
        bload(rb1, kchunk(1));
    } else {
        bload(rb1, kchunk(0));
    }
#pragma unroll
    for (int i = 0; i < H_LD; ++i) pro_row(0, i);
    hstore(0);
    if (BPF2) bstore(rb2, 0);
    else bstore(rb1, 0);
    __syncthreads();

#pragma unroll
    for (int cg = 0; cg < CG; ++cg) {
        f32x16 at[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) at[i][j][r] = 0.f;
        const bool more = cg + 1 < CG;
        // PRO (AZG_PRO_REMAT): the fragment row addresses are rebuilt per channel group
        // (a few VALU ops per tap) instead of 9 x 4 hoisted addresses living across the
        // unrolled groups -- with the prologue's registers those spilled, and every
        // reload's vmcnt wait drained the prefetch queue
        if constexpr (PRO != PRO_NONE && AZG_PRO_REMAT) {
#pragma unroll
            for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(hrow[i]));
        }
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int j = cg * 9 + tap;            // chunk index
            const int cur = j & 1;
            if (BPF2) {
                if (j + 2 < NCHK) bload(rb2, kchunk(j + 2));
            } else {
                if (j + 1 < NCHK) bload(rb1, kchunk(j + 1));
            }
            if (more && tap < H_LD) hload(cg + 1, tap);
            // keep the next chunk's global loads at the top of the chunk: without this
            // fence hipcc sinks them to just before their vmcnt wait (latency exposed)
            __builtin_amdgcn_sched_barrier(0);
            // split-fp16: the fragment addresses of each tap are built at the tap (a few
            // VALU ops) instead of 9 taps x 4 addresses hoisted and kept live across the
            // groups (round 5: that hoisting was the H3 towers' 96-336 B/lane of spills and
            // cost the per-layer H3 tile its second workgroup per CU).  Not in the fp32
            // bodies: measured slower there (fp32 tower 82.6 vs 87.2 % of peak at B = 512
            // spill-free, the fp32 train convs +50 us per step; scripts/gpu_r5ab.sh).
            if constexpr (H3 || AZG_EVAL_REMAT) {
#pragma unroll
                for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(hrow[i]), "+v"(vpix[i]));
            }
            const int d = (tap / 3 - 1) * PADW + (tap % 3 - 1);
            const int vd = (tap / 3 - 1) * BOARD + (tap % 3 - 1);
            int arow[TM], aswz[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = hrow[i] + d;
                arow[i] = r * BK;
                aswz[i] = VSWZ ? ((vpix[i] + vd) >> 1) & 7 : (r >> 1) & 7;
            }
            const float* Bb = Bs + cur * BN * BK;
            if constexpr (H3) {
#pragma unroll
                for (int st = 0; st < 2; ++st) {   // K16 steps: channels 16 st + 8 h + (0..7)
                    f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) {
                        ah[i] = *(const f16x8*)(Ah + arow[i] + (((2 * st + h) ^ aswz[i]) * 4));
                        al[i] = *(const f16x8*)(Ah + arow[i] + (((4 + 2 * st + h) ^ aswz[i]) * 4));
                    }
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        bh[j] = *(const f16x8*)(Bb + brow + j * 32 * BK + (((2 * st + h) ^ bswz) * 4));
                        bl[j] = *(const f16x8*)(Bb + brow + j * 32 * BK + (((4 + 2 * st + h) ^ bswz) * 4));
                    }
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j) {
                            // VAR bit 128 (train forward): the lo x lo term too -- products exact
                            // to ~2^-33, smallest first
                            if constexpr ((VAR & 128) != 0)
                                at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bl[j], at[i][j], 0, 0, 0);
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], at[i][j], 0, 0, 0);
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], at[i][j], 0, 0, 0);
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], at[i][j], 0, 0, 0);
                        }
                }
            } else
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 a[TM], b[TN];
                if (ABL & 8) {
#pragma unroll
                    for (int i = 0; i < TM; ++i) a[i] = rfix;
#pragma unroll
                    for (int j = 0; j < TN; ++j) b[j] = rfix;
                } else {
#pragma unroll
                    for (int i = 0; i < TM; ++i) a[i] = *(const f32x4*)(Ah + arow[i] + (((h * 4 + q) ^ aswz[i]) * 4));
                    const int rc = ((h * 4 + q) ^ bswz) * 4;
#pragma unroll
                    for (int j = 0; j < TN; ++j) b[j] = *(const f32x4*)(Bb + brow + j * 32 * BK + rc);
                }
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], at[i][j], 0, 0, 0);
            }
            // the row loaded one tap ago gets its BN / ReLU now (PRO)
            if (PRO != PRO_NONE && more && tap >= 1 && tap <= H_LD) pro_row(cg + 1, tap - 1);
            if (j + 1 < NCHK) {
                bstore(rb1, cur ^ 1);
                if (BPF2) {
#pragma unroll
                    for (int i = 0; i < B_LD; ++i) rb1[i] = rb2[i];
                }
            }
            if (!(ABL & 4)) __syncthreads();
            if (tap == 8 && more) {
                hstore(cg + 1);      // every wave is past its last read of this group's halo
                __syncthreads();
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] += at[i][j];
    }

    // the last chunk ended with a barrier: the staging buffers are free
    halo_epilogue<C, BN_, WM_, TM_, NW_, EPI, SC1, ABL, (VSWZ ? BN : BN + 8), (VAR & 8) != 0, XE,
                  (VAR & 16) ? 2 : (VAR & 32) ? 1 : 0>(
        acc, scale, shift, resid, out, out_rs, M, m0, n0, smem, ex, fx, H3 ? &guard : nullptr);
}

}  // namespace azg
