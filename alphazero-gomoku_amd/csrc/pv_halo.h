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

// LDS: halo rows [HR][32] + two weight chunks [2][BN][32]; the epilogue reuses it
// as a [BM][BN+8] tile.
template <int C, int BN, int WM, int TM, int NW>
constexpr int halo_lds_bytes()
{
    using T = ConvTile<C, BN, WM, TM, NW>;
    const int staging = ((halo_span(T::BM) + T::RPP - 1) / T::RPP * T::RPP + 2 * BN) * T::BK * 4;
    const int epilogue = T::BM * (BN + 8) * 4;
    return staging > epilogue ? staging : epilogue;
}

// Tower epilogue: BN scale/shift, residual added when `resid` is non-null, ReLU
// (EPI_BN_RELU / EPI_BN_RES_RELU chosen at run time, same arithmetic).
constexpr int EPI_BN_OPTRES_RELU = 4;

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
template <int C, int BN_, int WM_, int TM_, int NW_, int EPI, bool SC1 = false, int ABL = 0>
__device__ __forceinline__ void halo_tile(
    const float* __restrict__ in, const float* __restrict__ wp,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ resid, float* __restrict__ out, __amdgpu_buffer_rsrc_t out_rs,
    int M, int m0, int n0, float* smem)
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    constexpr int RPP = T::RPP;
    constexpr int BM = T::BM, BN = T::BN, BK = T::BK;
    constexpr int CG = T::CG, WN = T::WN, TM = T::TM, TN = T::TN;
    constexpr int B_LD = T::B_LD;
    constexpr int HS = halo_span(BM);
    constexpr int H_LD = (HS + RPP - 1) / RPP;
    constexpr int HR = H_LD * RPP;
    static_assert(RPP % 16 == 0, "halo staging rows must keep the row swizzle");
    static_assert(H_LD <= 9, "halo loads are spread over the 9 taps");

    float* Ah = smem;                 // [HR][32]
    float* Bs = smem + HR * BK;       // [2][BN][32]

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

    f32x4 rh[H_LD], rb[B_LD];
    auto hload = [&](int cg, int i) {
        if (ABL & 2) return;
        rh[i] = *(const f32x4*)(in + hsrc[i] + cg * BK);
    };
    auto bload = [&](int kc) {
        if (ABL & 1) return;
        const float* wk = wsrc + (size_t)kc * C * BK;
#pragma unroll
        for (int i = 0; i < B_LD; ++i) rb[i] = *(const f32x4*)(wk + RPP * i * BK);
    };
    // 16-B chunk c of LDS row r is stored at chunk c ^ ((r >> 1) & 7): any 16
    // consecutive rows a ds_read_b128 lane group touches land on distinct slots.
    const int wchunk = ((tid & 7) ^ ((sr >> 1) & 7)) * 4;
    auto hstore = [&]() {
#pragma unroll
        for (int i = 0; i < H_LD; ++i) *(f32x4*)(Ah + (sr + RPP * i) * BK + wchunk) = rh[i];
    };
    auto bstore = [&](int buf) {
        float* b = Bs + buf * BN * BK;
#pragma unroll
        for (int i = 0; i < B_LD; ++i) *(f32x4*)(b + (sr + RPP * i) * BK + wchunk) = rb[i];
    };

    // Lane l of an MFMA step s uses K index h*16+s (h = l>>5) for both A and B, so
    // each lane's 16 A values and 16 B values of a chunk are contiguous in LDS.
    const int r32 = lane & 31, h = lane >> 5;
    // halo row of each fragment pixel (tail pixels clamp to the last valid one)
    int hrow[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) hrow[i] = pad_row(min(m0 + wm * TM * 32 + i * 32 + r32, M - 1)) - hbase;
    const int bswz = (r32 >> 1) & 7;
    const int brow = (wn * TN * 32 + r32) * BK;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
    for (int i = 0; i < H_LD; ++i) hload(0, i);
    bload(0);
    hstore();
    bstore(0);
    __syncthreads();

    for (int cg = 0; cg < CG; ++cg) {
        f32x16 at[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) at[i][j][r] = 0.f;
        const bool more = cg + 1 < CG;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int cur = (cg + tap) & 1;        // chunk index cg*9 + tap, parity
            if (tap < 8) bload((tap + 1) * CG + cg);
            else if (more) bload(cg + 1);
            if (more && tap < H_LD) hload(cg + 1, tap);
            // keep the next chunk's global loads at the top of the chunk: without this
            // fence hipcc sinks them to just before their vmcnt wait (latency exposed)
            __builtin_amdgcn_sched_barrier(0);
            const int d = (tap / 3 - 1) * PADW + (tap % 3 - 1);
            int arow[TM], aswz[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = hrow[i] + d;
                arow[i] = r * BK;
                aswz[i] = (r >> 1) & 7;
            }
            const float* Bb = Bs + cur * BN * BK;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 a[TM], b[TN];
                if (ABL & 8) {
#pragma unroll
                    for (int i = 0; i < TM; ++i) a[i] = f32x4{(float)cg, (float)q, (float)i, (float)tap};
#pragma unroll
                    for (int j = 0; j < TN; ++j) b[j] = f32x4{(float)q, (float)cg, 1.f, (float)j};
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
            if (tap < 8 || more) bstore(cur ^ 1);
            if (!(ABL & 4)) __syncthreads();
            if (tap == 8 && more) {
                hstore();            // every wave is past its last read of this group's halo
                __syncthreads();
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] += at[i][j];
    }

    // Epilogue through LDS: the accumulators (C/D map of the 32x32 MFMA: col =
    // lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)) are written to an LDS tile
    // [BM][BN+8] (the +8 puts rows 4 apart on opposite bank halves: conflict-free),
    // then every thread finishes 16-B runs of 4 channels of one pixel: one pad_off,
    // float4 scale/shift/residual, one 16-B store per run -- instead of 16 scalar
    // stores (and 16 pad_off divisions) per fragment.  Same per-element arithmetic.
    constexpr int ELD = BN + 8;
    float* Es = smem;   // the last chunk ended with a barrier: staging buffers are free
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
    constexpr int CPR = BN / 4;            // 16-B runs per pixel row
    constexpr int RPI = T::NT / CPR;       // pixel rows per pass
    static_assert(BM % RPI == 0, "epilogue passes");
    const int ec = (tid % CPR) * 4;
    const int er = tid / CPR;
    const int col = n0 + ec;
    f32x4 s4 = {1.f, 1.f, 1.f, 1.f}, t4 = {0.f, 0.f, 0.f, 0.f};
    if (EPI == EPI_BN_RELU || EPI == EPI_BN_RES_RELU || EPI == EPI_BN_OPTRES_RELU) {
        s4 = *(const f32x4*)(scale + col);
        t4 = *(const f32x4*)(shift + col);
    }
#pragma unroll
    for (int p = 0; p < BM / RPI; ++p) {
        const int row = er + p * RPI;
        const int m = m0 + row;
        f32x4 v = *(const f32x4*)(Es + row * ELD + ec);
        if (m < M && (!(ABL & 16) || v[0] == 1234.5f)) {
            const int o = pad_off(m, C) + col;
            f32x4 rv = {0.f, 0.f, 0.f, 0.f};
            const bool has_res = EPI == EPI_BN_RES_RELU || EPI == EPI_ADD || (EPI == EPI_BN_OPTRES_RELU && resid);
            if (has_res) rv = *(const f32x4*)(resid + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = v[e];
                if (EPI == EPI_BN_RELU) {
                    x = fmaxf(x * s4[e] + t4[e], 0.f);
                } else if (EPI == EPI_BN_RES_RELU) {
                    x = fmaxf(x * s4[e] + t4[e] + rv[e], 0.f);
                } else if (EPI == EPI_BN_OPTRES_RELU) {
                    x = has_res ? fmaxf(x * s4[e] + t4[e] + rv[e], 0.f) : fmaxf(x * s4[e] + t4[e], 0.f);
                } else if (EPI == EPI_ADD) {
                    x = x + rv[e];
                }
                v[e] = x;
            }
            if constexpr (SC1) {
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), out_rs, o * 4, 0, 16);
            } else {
                *(f32x4*)(out + o) = v;
            }
        }
    }
}

}  // namespace azg
