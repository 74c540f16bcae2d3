// Split-fp16 (H3) eval conv tile, round 5 form: the same products and the same
// per-element K order as halo_tile's H3 body (pv_halo.h VAR bit 64, so the two are
// bitwise equal), restructured for what bounds that body on gfx950 -- the LDS.
//
// With three fp16 MFMAs per fp32-equivalent product the MFMA work per tap is 5.3x
// smaller than the fp32 tile's while the LDS operand bytes per tap are the same: the
// 32x32-per-wave body reads 1.33 KB of fragments per MFMA and stages its weights through
// registers and ds_write (the slow VGPR->LDS path), one barrier per tap, LDS-array busy
// 75 % at 54 % MFMA busy (scripts/h3_lab.hip, scripts/gpu_r5n.sh).  Here:
//  * the wave tile is TM x TN fragments of 32x32 (2x2: a 64x64 wave tile reads 0.67 KB
//    per MFMA -- every A fragment serves TN MFMA triples, every B fragment TM);
//  * weights reach LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows of one
//    chunk per wave-instruction, slot swizzle applied on the SOURCE address), NWB stage
//    buffers of TPS taps each, counted vmcnt waits and a raw s_barrier per stage (a
//    __syncthreads fence would drain the DMA in flight);
//  * halo rows stay register-staged (they are split into hi / lo while staged), loads
//    spread over the stages of the previous channel group, the board-keyed 16-B slot
//    swizzle (conflict-free fragment reads across board-row ends).
// Numerics: identical to halo_tile<..., VAR 99> (tested bitwise in the lab and by the
// GPU tests through every eval path).
#pragma once
#include "pv_halo.h"

namespace azg {

template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB>
struct H3Tile {
    using T = ConvTile<C, BN, WM, TM, NW>;
    static constexpr int BM = T::BM, BK = 32, CG = C / 32, WN = T::WN, TN = T::TN, RPP = T::RPP;
    static constexpr int HS = halo_span(BM);
    static constexpr int H_LD = (HS + RPP - 1) / RPP;
    static constexpr int HR = H_LD * RPP;
    static constexpr int NST = 9 / TPS;          // weight stages per channel group
    static constexpr int NSTAGE = CG * NST;
    static constexpr int PPS = TPS * BN / 8;     // 1-KiB weight pieces per stage
    static constexpr int PPW = PPS / NW;         // ... per wave
    static constexpr int STAGING = (HR + NWB * TPS * BN) * BK * 4;
    static constexpr int EPI_BYTES = BM * BN * 4;
    static constexpr int PROW_OFF = STAGING > EPI_BYTES ? STAGING : EPI_BYTES;   // [BM] pad rows (direct epilogue)
    static constexpr int LDS = PROW_OFF;              // + BM * 4 with the direct epilogue (h3_lds_bytes)
    static_assert(9 % TPS == 0, "stages hold whole taps");
    static_assert(PPS % NW == 0, "every wave issues the same weight pieces (counted waits)");
    static_assert(NWB >= 2 && NWB <= 3, "two or three weight stage buffers");
    static_assert(RPP % 16 == 0, "halo staging rows keep the row swizzle");
};

// OPT bits (tile-body options, all bitwise identical): 8 = every halo row of the next
// channel group is loaded at the group's first stage (else row i at stage i % NST);
// 16 = the epilogue issues its residual / scale / shift loads before the LDS pass;
// 32 = direct epilogue: every lane finishes its own accumulators (4-B loads / stores in
// the MFMA C layout, pad rows from a per-tile LDS table) -- no LDS pass, no barrier.
// The stage (within a group) at which halo row i of the next group is loaded:
constexpr int h3_halo_stage(int i, int nst, int opt) { return (opt & 8) ? 0 : i % nst; }
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int OPT>
constexpr int h3_lds_bytes()
{
    using H = H3Tile<C, BN, WM, TM, NW, TPS, NWB>;
    return H::LDS + ((OPT & 32) ? H::BM * 4 : 0);
}
// halo loads of stage s (global stage index): rows of the NEXT channel group (none in
// the last group)
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int OPT>
constexpr int h3_halo_loads(int s)
{
    using H = H3Tile<C, BN, WM, TM, NW, TPS, NWB>;
    if (s < 0 || s >= H::NSTAGE || s / H::NST + 1 >= H::CG) return 0;
    int n = 0;
    for (int i = 0; i < H::H_LD; ++i) n += h3_halo_stage(i, H::NST, OPT) == (s % H::NST);
    return n;
}
// weight pieces a wave issues at the top of stage s (those of stage s + NWB - 1)
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB>
constexpr int h3_dma_pieces(int s)
{
    using H = H3Tile<C, BN, WM, TM, NW, TPS, NWB>;
    return (s >= 0 && s + NWB - 1 < H::NSTAGE) ? H::PPW : 0;
}
// vector-memory operations a wave issued after the last weight piece of stage s + 1,
// up to and including the top of stage s: the vmcnt that retires stage s + 1's weights
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int OPT>
constexpr int h3_wait_next(int s)
{
    const int t = s + 1 - (NWB - 1);   // the stage whose top issued stage s + 1's pieces
    int n = h3_halo_loads<C, BN, WM, TM, NW, TPS, NWB, OPT>(t);
    for (int u = t + 1; u <= s; ++u)
        n += h3_dma_pieces<C, BN, WM, TM, NW, TPS, NWB>(u) + h3_halo_loads<C, BN, WM, TM, NW, TPS, NWB, OPT>(u);
    return n;
}
// vector-memory operations issued after the last halo load of group g (through the top
// of the group's last stage): the vmcnt that retires the halo registers
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int OPT>
constexpr int h3_wait_halo(int g)
{
    using H = H3Tile<C, BN, WM, TM, NW, TPS, NWB>;
    int last = -1;
    for (int s = g * H::NST; s < (g + 1) * H::NST; ++s)
        if (h3_halo_loads<C, BN, WM, TM, NW, TPS, NWB, OPT>(s)) last = s;
    if (last < 0) return 0;
    int n = 0;
    for (int u = last + 1; u < (g + 1) * H::NST; ++u)
        n += h3_dma_pieces<C, BN, WM, TM, NW, TPS, NWB>(u) + h3_halo_loads<C, BN, WM, TM, NW, TPS, NWB, OPT>(u);
    return n;
}

// s_waitcnt vmcnt(n) for a value the unrolled loop folds to a constant
__device__ __forceinline__ void h3_wait_vm(int n)
{
#define AZG_H3_VM(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n <= 0 ? 0 : n >= 15 ? 15 : n) {
        AZG_H3_VM(0) AZG_H3_VM(1) AZG_H3_VM(2) AZG_H3_VM(3) AZG_H3_VM(4) AZG_H3_VM(5) AZG_H3_VM(6) AZG_H3_VM(7)
        AZG_H3_VM(8) AZG_H3_VM(9) AZG_H3_VM(10) AZG_H3_VM(11) AZG_H3_VM(12) AZG_H3_VM(13) AZG_H3_VM(14)
        AZG_H3_VM(15)
    }
#undef AZG_H3_VM
}
__device__ __forceinline__ void h3_raw_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
}

// One BM x BN output tile at (m0, n0) of a split-fp16 residual conv (eval epilogue).
// wp: the pack_h3 weights ([tap * C/32 + cg][cout][hi 32 | lo 32] halves); scale: the
// H3 BN scale (carries the weights' power-of-two scaling).  RBUF: residual read form
// (halo_epilogue).  LDS: H3Tile::LDS bytes at smem.
// ABL (timing studies only, results invalid when set): bit 1 skips the epilogue (a
// never-true compare keeps the accumulators live), bit 2 the halo loads, bit 4 the
// weight DMA.
template <int C, int BN_, int WM_, int TM_, int NW_, int TPS, int NWB, int EPI, bool SC1, int RBUF, int ABL = 0,
          int OPT = 0>
__device__ __forceinline__ void h3_tile(const float* __restrict__ in, const float* __restrict__ wp,
                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                        const float* __restrict__ resid, float* __restrict__ out,
                                        __amdgpu_buffer_rsrc_t out_rs, int M, int m0, int n0, float* smem,
                                        const H3Guard& guard)
{
    using H = H3Tile<C, BN_, WM_, TM_, NW_, TPS, NWB>;
    using T = typename H::T;
    constexpr int BM = H::BM, BN = BN_, BK = 32, CG = H::CG, WN = H::WN, TM = TM_, TN = H::TN, NW = NW_;
    constexpr int RPP = H::RPP, H_LD = H::H_LD, HR = H::HR, NST = H::NST, NSTAGE = H::NSTAGE;
    constexpr int PPW = H::PPW, BNP = BN / 8;   // weight pieces per tap
    static_assert(C % BN == 0, "N tiles");

    float* Ah = smem;                 // [HR][32]: split halo rows
    float* Bs = smem + HR * BK;       // [NWB][TPS][BN][32]: split weight rows
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int mlast = min(m0 + BM, M) - 1;
    const int hbase = pad_row(m0) - (PADW + 1);
    const int hmax = pad_row(mlast) + (PADW + 1);

    if constexpr ((OPT & 32) != 0) {   // pad rows of the tile's pixels (-1: past the batch)
        int* prow = (int*)(smem + H::PROW_OFF / 4);
        for (int p = tid; p < BM; p += T::NT) prow[p] = m0 + p < M ? pad_row(m0 + p) : -1;
    }

    // ---- halo staging (registers; split while stored) ----
    const int sr = tid >> 3, sc = (tid & 7) * 4;
    int hsrc[H_LD], hkey[H_LD];
#pragma unroll
    for (int i = 0; i < H_LD; ++i) {
        const int r = min(hbase + sr + RPP * i, hmax);
        hsrc[i] = (r * C + sc) * 4;
        hkey[i] = (halo_vkey(hbase + sr + RPP * i) >> 1) & 7;
    }
    const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), (short)0,
                                                                          0x7fffffff, 0x00020000);
    f32x4 rh[H_LD];
    auto hload = [&](int g, int i) {
        if (ABL & 2) return;
        rh[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, hsrc[i] + g * BK * 4, 0, 0));
    };
    auto hstore = [&]() {
        const int q = (tid & 7) >> 1, half = (tid & 1) * 2;
#pragma unroll
        for (int i = 0; i < H_LD; ++i) {
            f16x4 hi, lo;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                hi[e] = (_Float16)rh[i][e];
                lo[e] = (_Float16)(rh[i][e] - (float)hi[e]);
            }
            float* row = Ah + (sr + RPP * i) * BK;
            *(f16x4*)(row + ((q ^ hkey[i]) * 4) + half) = hi;
            *(f16x4*)(row + (((4 + q) ^ hkey[i]) * 4) + half) = lo;
        }
    };

    // ---- weight pieces (LDS-DMA) ----
    // piece p of a stage: tap p / BNP of the stage, rows 8 (p % BNP) .. +7; lane: row + lane/8,
    // LDS slot lane%8 holding source chunk slot ^ key(row)
    const int lr = lane >> 3, ls = lane & 7;
    int woff[PPW], wdst[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int p = wid + NW * i;
        const int tt = p / BNP, row = (p % BNP) * 8 + lr;
        woff[i] = tt * C * BK * CG + (n0 + row) * BK + ((ls ^ ((row >> 1) & 7)) * 4);   // + stage base
        wdst[i] = (tt * BN + (p % BNP) * 8) * BK;                                          // + buffer base
    }
    auto dma_stage = [&](int s) {   // stage s = channel group s / NST, taps TPS (s % NST) ..
        if (ABL & 4) return;
        const int g = s / NST, t0 = (s % NST) * TPS;
        const float* src = wp + (size_t)(t0 * CG + g) * C * BK;
        float* dst = Bs + (s % NWB) * TPS * BN * BK;
#pragma unroll
        for (int i = 0; i < PPW; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + woff[i]),
                                             (__attribute__((address_space(3))) void*)(dst + wdst[i]), 16, 0, 0);
    };

    // ---- fragments ----
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

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // prologue: weights of the first NWB - 1 stages, the first group's halo
#pragma unroll
    for (int s = 0; s < NWB - 1; ++s)
        if (s < NSTAGE) dma_stage(s);
#pragma unroll
    for (int i = 0; i < H_LD; ++i) hload(0, i);
    if (ABL & 2) {
#pragma unroll
        for (int i = 0; i < H_LD; ++i) rh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    h3_wait_vm(0);
    hstore();
    h3_raw_barrier();

#pragma unroll
    for (int cg = 0; cg < CG; ++cg) {
        f32x16 at[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) at[i][j][r] = 0.f;
#pragma unroll
        for (int sg = 0; sg < NST; ++sg) {
            const int s = cg * NST + sg;
            if (s + NWB - 1 < NSTAGE) dma_stage(s + NWB - 1);
            // the counted waits assume this issue order (weights, then halo rows): keep
            // the scheduler from hoisting the halo loads above the DMA
            __builtin_amdgcn_sched_barrier(0);
            if (cg + 1 < CG) {
#pragma unroll
                for (int i = 0; i < H_LD; ++i)
                    if (h3_halo_stage(i, NST, OPT) == sg) hload(cg + 1, i);
            }
            __builtin_amdgcn_sched_barrier(0);
            const float* Bst = Bs + (s % NWB) * TPS * BN * BK;
#pragma unroll
            for (int tt = 0; tt < TPS; ++tt) {
                const int tap = sg * TPS + tt;
                // the tap's fragment addresses are built here (not hoisted across groups)
#pragma unroll
                for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(hrow[i]), "+v"(vpix[i]));
                const int d = (tap / 3 - 1) * PADW + (tap % 3 - 1);
                const int vd = (tap / 3 - 1) * BOARD + (tap % 3 - 1);
                int arow[TM], aswz[TM];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    arow[i] = (hrow[i] + d) * BK;
                    aswz[i] = ((vpix[i] + vd) >> 1) & 7;
                }
                const float* Bb = Bst + tt * BN * BK;
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
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], at[i][j], 0, 0, 0);
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], at[i][j], 0, 0, 0);
                            at[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], at[i][j], 0, 0, 0);
                        }
                }
            }
            // retire stage s + 1's weights (what was issued after them may stay in flight);
            // every wave is then past its reads of stage s's buffer and of this group's halo
            h3_wait_vm(s + 1 < NSTAGE ? h3_wait_next<C, BN_, WM_, TM_, NW_, TPS, NWB, OPT>(s) : 0);
            h3_raw_barrier();
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] += at[i][j];
        if (cg + 1 < CG) {
            h3_wait_vm(h3_wait_halo<C, BN_, WM_, TM_, NW_, TPS, NWB, OPT>(cg));
            hstore();
            h3_raw_barrier();
        }
    }

    // the last stage ended with a barrier: the staging buffers are free for the epilogue
    if constexpr ((ABL & 1) != 0) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) v += acc[i][j][r];
        if (v == 1234.5f) out[tid] = v;
        return;
    }
    if constexpr ((OPT & 32) != 0) {
        __builtin_amdgcn_sched_barrier(0);
        const int* prow = (const int*)(smem + H::PROW_OFF / 4);
        const bool has_res = EPI == EPI_BN_RES_RELU || (EPI == EPI_BN_OPTRES_RELU && resid);
        const __amdgpu_buffer_rsrc_t res_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(resid), (short)0,
                                                                               0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t out_ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
        bool bad = false;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * TN * 32 + j * 32 + r32;
            const float sj = scale[col], tj = shift[col];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                int pr[16];
                float rv[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int4 p4 = *(const int4*)(prow + wm * TM * 32 + i * 32 + 8 * q + 4 * h);
                    pr[4 * q] = p4.x, pr[4 * q + 1] = p4.y, pr[4 * q + 2] = p4.z, pr[4 * q + 3] = p4.w;
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    rv[r] = 0.f;
                    if (has_res && pr[r] >= 0) {
                        const int o = pr[r] * C + col;
                        rv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(res_rs, o * 4, 0,
                                                                                               RBUF == 2 ? 16 : 0));
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float x = acc[i][j][r];
                    bad |= !__builtin_isfinite(x);
                    // the halo_epilogue arithmetic, element for element
                    const float y = has_res ? fmaxf(fmaf(x, sj, tj) + rv[r], 0.f) : fmaxf(fmaf(x, sj, tj), 0.f);
                    // 32-bit offsets into one buffer resource (64-bit addresses per store spill)
                    if (pr[r] >= 0)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), out_ws, (pr[r] * C + col) * 4,
                                                              0, SC1 ? 16 : 0);
                }
                // one fragment's loads in flight at a time (hoisting every fragment's 16
                // residual loads above the first store spills)
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (bad && guard.ring && guard.seq)
            __hip_atomic_store(guard.ring + (guard.seq & (kH3RingSize - 1)), guard.seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    halo_epilogue<C, BN_, WM_, TM_, NW_, EPI, SC1, 0, BN, (OPT & 16) != 0, XE_NONE, RBUF>(acc, scale, shift, resid, out, out_rs,
                                                                                 M, m0, n0, smem, EpiX{}, FinX{}, &guard);
}

}  // namespace azg
