// Weight-gradient tile of the 3x3 convolution and its slab reduction (pv_wgrad.hip).
//   dW[co][ci][tap] = sum_m dz[m][co] * X[m + off(tap)][ci]   (autograd of network.py:12,14)
#pragma once
#include "pv_common.h"

namespace azg {

// Split s covers the whole 32-pixel chunks [s*NCH/S, (s+1)*NCH/S) of the batch
// (NCH = ceil(M/32)).  Rows past M load zeros.
__device__ __forceinline__ void wgrad_split_rows(int split, int S, int M, int& mbeg, int& mend)
{
    const int nch = (M + 31) / 32;
    mbeg = (int)((int64_t)split * nch / S) * 32;
    mend = min(M, (int)((int64_t)(split + 1) * nch / S) * 32);
}

// Geometry of the LDS-DMA weight-grad tile: BT x BT outputs (co x ci) of one tap, K =
// the pixels of one split in chunks of 32.  NWV = 4: 2 x 2 waves of (BT/2)^2; NWV = 8
// (BT = 128): 2 x 4 waves of 64 co x 32 ci.  Both give every output the same chain.
template <int C>
struct WgNat {
    static constexpr int BT = C < 128 ? C : 128;
    static constexpr int NT = C / BT;               // tiles per edge
    static constexpr int TILES = 9 * NT * NT;       // tiles per pixel split
    static constexpr int LDS_BYTES = 2 * 2 * 32 * BT * 4;
    static constexpr int NWV = BT >= 128 ? 8 : 4;   // waves of an 8-wave workgroup that work
};

// One weight-grad tile (split, tap, co0, ci0) with NATURAL operand rows in LDS filled
// by LDS-DMA: each wave-instruction global_load_lds_dwordx4 moves 1 KiB = 256/BT pixel
// rows of BT channels straight into LDS (no staging VGPRs, no ds_write), issued one chunk
// ahead.  MFMA step s reads, per operand, one ds_read_b32 per lane: lanes 0-31 pixel s,
// lanes 32-63 pixel s + 16, 32 consecutive channels.  16-B chunk j of LDS row p holds
// global chunk j ^ 8*((p >> 4) & 1) (swizzle on each lane's source address,
// cdna_hip_programming.md §5.4): the two half-waves of a fragment read land on disjoint
// bank halves.  Rows past the split read padded pixel 0 (the zero halo).
// Waves wid >= NWV of a larger workgroup only join the barriers.  The caller guarantees
// every wave is past its last read of `smem` (barrier) before the call; the call ends
// with the slab stores issued (not drained).
template <int C, bool WT, int NWV>
__device__ __forceinline__ void wgrad_nat_tile(const float* __restrict__ dz, const float* __restrict__ x,
                                               float* __restrict__ slab, int M, int S, int split, int tap,
                                               int co0, int ci0, float* smem)
{
    constexpr int BT = C < 128 ? C : 128, BK = 32;
    constexpr int WNW = NWV == 8 ? 4 : 2;           // waves along ci
    constexpr int TA = BT / 64, TB = BT / (32 * WNW); // accumulators along co / ci per wave
    constexpr int RPI = 256 / BT;      // pixel rows per wave-instruction (1 KiB)
    constexpr int CPR = BT / 4;        // 16-B chunks per row
    constexpr int IPW = BK / RPI / NWV;  // instructions per wave per operand per chunk
    static_assert(IPW >= 1 && CPR >= 16 && TB >= 1, "tile");
    float* As = smem;                  // [2][BK][BT]  dz rows (co)
    float* Bs = smem + 2 * BK * BT;    // [2][BK][BT]  x rows (ci, tap-shifted)

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bool active = wid < NWV;
    const int wm = wid / WNW, wn = wid % WNW;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    int mbeg, mend;
    wgrad_split_rows(split, S, M, mbeg, mend);
    const int nch = (mend - mbeg + BK - 1) / BK;

    auto glds = [](const float* src, float* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    const int ri = lane / CPR, jl = lane % CPR;
    auto issue = [&](int kc, int buf) {
        if (!active) return;
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int r0 = (wid * IPW + i) * RPI;       // first LDS row of this instruction
            const int p = r0 + ri;
            const int m = mbeg + kc * BK + p;
            const int j = jl ^ (((p >> 4) & 1) << 3);
            const int po = m < mend ? pad_off(m, C) : 0;
            const int px = m < mend ? po + toff : 0;
            glds(dz + po + co0 + 4 * j, As + buf * BK * BT + r0 * BT);
            glds(x + px + ci0 + 4 * j, Bs + buf * BK * BT + r0 * BT);
        }
    };
    const int r32 = lane & 31, h = lane >> 5;
    int aoff[TA], boff[TB];
#pragma unroll
    for (int i = 0; i < TA; ++i) {
        const int ca = wm * (BT / 2) + i * 32 + r32;
        aoff[i] = 16 * h * BT + (((ca >> 2) ^ (h << 3)) << 2) + (ca & 3);
    }
#pragma unroll
    for (int j = 0; j < TB; ++j) {
        const int cb = wn * (BT / WNW) + j * 32 + r32;
        boff[j] = 16 * h * BT + (((cb >> 2) ^ (h << 3)) << 2) + (cb & 3);
    }

    f32x16 acc[TA][TB];
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    if (nch > 0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kc = 0; kc < nch; ++kc) {
        const int cur = kc & 1;
        // the other buffer's last reads ended at the previous chunk's barrier
        if (kc + 1 < nch) issue(kc + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        if (active) {
            const float* Ab = As + cur * BK * BT;
            const float* Bb = Bs + cur * BK * BT;
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                float a[TA], b[TB];
#pragma unroll
                for (int i = 0; i < TA; ++i) a[i] = Ab[s * BT + aoff[i]];
#pragma unroll
                for (int j = 0; j < TB; ++j) b[j] = Bb[s * BT + boff[j]];
#pragma unroll
                for (int i = 0; i < TA; ++i)
#pragma unroll
                    for (int j = 0; j < TB; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of chunk kc+1 retired
        __syncthreads();
    }

    if (active) {
        float* out = slab + ((size_t)split * 9 + tap) * C * C;
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, (size_t)C * C * sizeof(float));
#pragma unroll
        for (int i = 0; i < TA; ++i)
#pragma unroll
            for (int j = 0; j < TB; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = co0 + wm * (BT / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int ci = ci0 + wn * (BT / WNW) + j * 32 + r32;
                    store1<WT>(out, rs, co * C + ci, acc[i][j][r]);
                }
    }
}

// Round-5 form of the same tile (wgrad_nat_tile2): identical MFMA sequence per output
// element (same splits, chunks, steps and pixel -> K-lane map, so the slabs are bitwise
// those of wgrad_nat_tile), with the per-row address arithmetic taken out of the chunk
// loop (VALU/MFMA 2.74, the highest of any conv):
//  * the padded row of every pixel comes from a table built once per workspace
//    (rowtab[m] = pad_row(m)), loaded two chunks ahead -- one buffer_load_dword per
//    staged row instead of the divisions by 225 and 15 of pad_off;
//  * operands reach LDS by buffer_load ... lds (LDS-DMA through a buffer resource): one
//    32-bit voffset per row serves both operands (the x resource's base is shifted by
//    the tap's row offset), no 64-bit address arithmetic;
//  * rows past the batch (a partial last chunk) are read past num_records: zeros;
//  * the slab keeps the MFMA C/D layout (slab_mfma_index): 16-B stores, 16 per lane
//    instead of 64 4-B stores; wgrad_reduce_mfma sums it in wgrad_reduce_elems' order.
constexpr int kRowTabPad = 64;   // rowtab entries past M (never read: rows >= M are predicated)
template <int C, int NWV>
struct WgMfmaLayout {
    static constexpr int BT = C < 128 ? C : 128;
    static constexpr int NT = C / BT;
    static constexpr int WNW = NWV == 8 ? 4 : 2;
    static constexpr int TA = BT / 64, TB = BT / (32 * WNW);
    // float index inside one tap's C*C block of the slab of C/D register r = 4q + e of
    // `lane`: one 16-B store instruction (fixed q) writes 1 KiB contiguous per wave
    __host__ __device__ static constexpr int index(int tco, int tci, int w, int i, int j, int lane, int r)
    {
        return ((((((tco * NT + tci) * NWV + w) * TA + i) * TB + j) * 4 + (r >> 2)) * 64 + lane) * 4 + (r & 3);
    }
};
template <int C, bool WT, int NWV>
__device__ __forceinline__ void wgrad_nat_tile2(const float* __restrict__ dz, const float* __restrict__ x,
                                                const int* __restrict__ rowtab, float* __restrict__ slab, int M,
                                                int S, int split, int tap, int co0, int ci0, float* smem)
{
    constexpr int BT = C < 128 ? C : 128, BK = 32;
    using L = WgMfmaLayout<C, NWV>;
    constexpr int WNW = L::WNW, TA = L::TA, TB = L::TB;
    constexpr int RPI = 256 / BT;      // pixel rows per wave-instruction (1 KiB)
    constexpr int CPR = BT / 4;        // 16-B chunks per row
    constexpr int IPW = BK / RPI / NWV;  // instructions per wave per operand per chunk
    constexpr int LC = C == 64 ? 8 : C == 128 ? 9 : 10;   // log2(C * 4): bytes per padded row
    static_assert((1 << LC) == C * 4, "row shift");
    static_assert(IPW >= 1 && CPR >= 16 && TB >= 1, "tile");
    float* As = smem;                  // [2][BK][BT]  dz rows (co)
    float* Bs = smem + 2 * BK * BT;    // [2][BK][BT]  x rows (ci, tap-shifted)

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bool active = wid < NWV;
    const int wm = wid / WNW, wn = wid % WNW;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    int mbeg, mend;
    wgrad_split_rows(split, S, M, mbeg, mend);
    const int nch = (mend - mbeg + BK - 1) / BK;
    const int bytes = (int)padded_bytes(M, C);
    // x's resource starts at the tap's row shift: one voffset addresses both operands
    // (interior rows shifted by a tap stay inside the tensor)
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dz), (short)0, bytes,
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + toff), (short)0,
                                                                         bytes - toff * 4, 0x00020000);
    const int ri = lane / CPR, jl = lane % CPR;
    int colb[IPW];   // byte offset of this lane's 16-B column chunk, per instruction
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
        const int p = (wid * IPW + i) * RPI + ri;
        colb[i] = (co0 + 4 * (jl ^ (((p >> 4) & 1) << 3))) * 4;
    }
    const int colx = (ci0 - co0) * 4;   // x columns start at ci0
    // padded rows of this lane's pixels of chunk kc (two chunks in flight in registers)
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(rowtab), (short)0, M * 4,
                                                                         0x00020000);
    // the raw table rows of chunk kc (validity is applied when they are consumed, so no
    // wait on these loads is placed before the chunk's MFMAs)
    auto rows = [&](int kc, int (&r)[IPW]) {
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int m = mbeg + kc * BK + (wid * IPW + i) * RPI + ri;
            r[i] = (int)__builtin_amdgcn_raw_buffer_load_b32(rt, m * 4, 0, 0);   // past M: 0 (masked in issue)
        }
    };
    auto issue = [&](const int (&r)[IPW], int kc, int buf) {
        if (!active) return;
        const bool part = mbeg + (kc + 1) * BK > mend;   // wave-uniform: the split's partial last chunk
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int r0 = (wid * IPW + i) * RPI;       // first LDS row of this instruction
            int vo = (r[i] << LC) + colb[i], vx = vo + colx;
            if (part && mbeg + kc * BK + r0 + ri >= mend) {   // past the split: read past num_records = zeros
                vo = 0x7ffffff0;
                vx = 0x7ffffff0;
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (__attribute__((address_space(3))) void*)(As + buf * BK * BT + r0 * BT),
                                                     16, vo, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(Bs + buf * BK * BT + r0 * BT),
                                                     16, vx, 0, 0, 0);
        }
    };
    const int r32 = lane & 31, h = lane >> 5;
    int aoff[TA], boff[TB];
#pragma unroll
    for (int i = 0; i < TA; ++i) {
        const int ca = wm * (BT / 2) + i * 32 + r32;
        aoff[i] = 16 * h * BT + (((ca >> 2) ^ (h << 3)) << 2) + (ca & 3);
    }
#pragma unroll
    for (int j = 0; j < TB; ++j) {
        const int cb = wn * (BT / WNW) + j * 32 + r32;
        boff[j] = 16 * h * BT + (((cb >> 2) ^ (h << 3)) << 2) + (cb & 3);
    }

    f32x16 acc[TA][TB];
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // table rows of the chunks in flight, two register slots: slot (kc & 1) holds the rows
    // of chunk kc; at chunk kc the slot of chunk kc + 1 is consumed by its DMA issue and
    // refilled with chunk kc + 3's rows.  The loop is unrolled by two so the slots never
    // move between registers (a loop-carried copy would wait on the fresh loads).
    int ra[IPW], rb[IPW];
    if (active && nch > 0) {
        rows(0, ra);
        if (nch > 1) rows(1, rb);
        issue(ra, 0, 0);
        if (nch > 2) rows(2, ra);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    auto chunk = [&](int kc, int (&rnext)[IPW]) {
        const int cur = kc & 1;
        // the other buffer's last reads ended at the previous chunk's barrier
        if (kc + 1 < nch) {
            issue(rnext, kc + 1, cur ^ 1);
            if (active && kc + 3 < nch) rows(kc + 3, rnext);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (active) {
            const float* Ab = As + cur * BK * BT;
            const float* Bb = Bs + cur * BK * BT;
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                float a[TA], b[TB];
#pragma unroll
                for (int i = 0; i < TA; ++i) a[i] = Ab[s * BT + aoff[i]];
#pragma unroll
                for (int j = 0; j < TB; ++j) b[j] = Bb[s * BT + boff[j]];
#pragma unroll
                for (int i = 0; i < TA; ++i)
#pragma unroll
                    for (int j = 0; j < TB; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of chunk kc+1 retired
        __syncthreads();
    };
    for (int kc = 0; kc < nch; kc += 2) {
        chunk(kc, rb);                   // chunk kc + 1 (odd) lives in rb
        if (kc + 1 < nch) chunk(kc + 1, ra);
    }

    if (active) {
        float* out = slab + ((size_t)split * 9 + tap) * C * C;
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, (size_t)C * C * sizeof(float));
        const int tco = co0 / BT, tci = ci0 / BT;
#pragma unroll
        for (int i = 0; i < TA; ++i)
#pragma unroll
            for (int j = 0; j < TB; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
                    store4<WT>(out, rs, L::index(tco, tci, wid, i, j, lane, 4 * q), v);
                }
    }
}

// The slab sum of wgrad_reduce_elems for the MFMA-layout slabs of wgrad_nat_tile2: a
// thread sums one float4 run (4 consecutive C/D registers r = 4q..4q+3 of one lane:
// 4 output channels co, one input channel ci) over the S slabs in the same per-element
// order -- slabs k = 0,1,2,3 mod 4 in four partial sums, ((p0 + p1) + (p2 + p3)) -- and
// scatters it into torch's [co][ci][3][3]: bitwise the dW of the v1 path.
template <int C, int NWV>
__device__ __forceinline__ void wgrad_reduce_mfma(const float* __restrict__ slab, float* __restrict__ dw, int S,
                                                  int f)
{
    using L = WgMfmaLayout<C, NWV>;
    constexpr int BT = L::BT;
    const int total4 = 9 * C * C / 4;
    if (f >= total4) return;
    const f32x4* s4 = (const f32x4*)slab;
    f32x4 p0 = {0.f, 0.f, 0.f, 0.f}, p1 = p0, p2 = p0, p3 = p0;
    int k = 0;
    for (; k + 4 <= S; k += 4) {
        const f32x4 a = s4[(size_t)k * total4 + f], b = s4[(size_t)(k + 1) * total4 + f];
        const f32x4 c = s4[(size_t)(k + 2) * total4 + f], d = s4[(size_t)(k + 3) * total4 + f];
        p0 += a;
        p1 += b;
        p2 += c;
        p3 += d;
    }
    if (k < S) p0 += s4[(size_t)k * total4 + f];
    if (k + 1 < S) p1 += s4[(size_t)(k + 1) * total4 + f];
    if (k + 2 < S) p2 += s4[(size_t)(k + 2) * total4 + f];
    const f32x4 r = (p0 + p1) + (p2 + p3);
    // decode the slab index of element 4f (e = 0; L::index)
    const int idx = 4 * f;
    const int tap = idx / (C * C);
    int rem = (idx - tap * C * C) >> 2;
    const int lane = rem & 63;
    rem >>= 6;
    const int rq = (rem & 3) * 4;      // r of the first element
    rem >>= 2;
    const int j = rem % L::TB;
    rem /= L::TB;
    const int i = rem % L::TA;
    rem /= L::TA;
    const int w = rem % NWV;
    const int t = rem / NWV;
    const int tco = t / L::NT, tci = t % L::NT;
    const int wm = w / L::WNW, wn = w % L::WNW;
    const int r32 = lane & 31, h = lane >> 5;
    const int ci = tci * BT + wn * (BT / L::WNW) + j * 32 + r32;
    const int cob = tco * BT + wm * (BT / 2) + i * 32 + 8 * (rq >> 2) + 4 * h;
#pragma unroll
    for (int e = 0; e < 4; ++e) dw[((cob + e) * C + ci) * 9 + tap] = r[e];
}

// dW (torch layout [co][ci][3][3]) element idx of the slab layout [tap][co][ci] = the S
// slabs summed in a fixed order: four interleaved partial sums (slabs k = 0,1,2,3 mod 4)
// combined as ((p0 + p1) + (p2 + p3)).  NV consecutive-by-`stride` elements per call,
// every slab's loads of them issued together (the per-element order is unchanged).
template <int NV>
__device__ __forceinline__ void wgrad_reduce_elems(const float* __restrict__ slab, float* __restrict__ dw, int C,
                                                   int S, int idx0, int stride)
{
    const int total = 9 * C * C;
    float p0[NV], p1[NV], p2[NV], p3[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) p0[v] = p1[v] = p2[v] = p3[v] = 0.f;
    int k = 0;
    for (; k + 4 <= S; k += 4) {
        float a[NV], b[NV], c[NV], d[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int idx = min(idx0 + v * stride, total - 1);
            a[v] = slab[(size_t)k * total + idx];
            b[v] = slab[(size_t)(k + 1) * total + idx];
            c[v] = slab[(size_t)(k + 2) * total + idx];
            d[v] = slab[(size_t)(k + 3) * total + idx];
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            p0[v] += a[v];
            p1[v] += b[v];
            p2[v] += c[v];
            p3[v] += d[v];
        }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int idx = idx0 + v * stride;
        if (idx >= total) continue;
        if (k < S) p0[v] += slab[(size_t)k * total + idx];
        if (k + 1 < S) p1[v] += slab[(size_t)(k + 1) * total + idx];
        if (k + 2 < S) p2[v] += slab[(size_t)(k + 2) * total + idx];
        const int tap = idx / (C * C);
        const int rem = idx - tap * C * C;
        const int co = rem / C, ci = rem - co * C;
        dw[(co * C + ci) * 9 + tap] = (p0[v] + p1[v]) + (p2[v] + p3[v]);
    }
}

// The same reduction, float4-wide: a thread sums NV4 runs of 4 consecutive slab
// elements (run v at float4 index f0 + v * stride4), every slab's loads of them issued
// together -- a quarter of wgrad_reduce_elems' load instructions for the same bytes.
// Per element the order is wgrad_reduce_elems' (slabs k = 0,1,2,3 mod 4 in four partial
// sums, ((p0 + p1) + (p2 + p3))): bitwise equal.
template <int NV4>
__device__ __forceinline__ void wgrad_reduce_vec4(const float* __restrict__ slab, float* __restrict__ dw, int C,
                                                  int S, int f0, int stride4)
{
    const int total4 = 9 * C * C / 4;
    const f32x4* s4 = (const f32x4*)slab;
    f32x4 p0[NV4], p1[NV4], p2[NV4], p3[NV4];
#pragma unroll
    for (int v = 0; v < NV4; ++v) p0[v] = p1[v] = p2[v] = p3[v] = f32x4{0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 4 <= S; k += 4) {
        f32x4 a[NV4], b[NV4], c[NV4], d[NV4];
#pragma unroll
        for (int v = 0; v < NV4; ++v) {
            const int f = min(f0 + v * stride4, total4 - 1);
            a[v] = s4[(size_t)k * total4 + f];
            b[v] = s4[(size_t)(k + 1) * total4 + f];
            c[v] = s4[(size_t)(k + 2) * total4 + f];
            d[v] = s4[(size_t)(k + 3) * total4 + f];
        }
#pragma unroll
        for (int v = 0; v < NV4; ++v) {
            p0[v] += a[v];
            p1[v] += b[v];
            p2[v] += c[v];
            p3[v] += d[v];
        }
    }
#pragma unroll
    for (int v = 0; v < NV4; ++v) {
        const int f = f0 + v * stride4;
        if (f >= total4) continue;
        if (k < S) p0[v] += s4[(size_t)k * total4 + f];
        if (k + 1 < S) p1[v] += s4[(size_t)(k + 1) * total4 + f];
        if (k + 2 < S) p2[v] += s4[(size_t)(k + 2) * total4 + f];
        const f32x4 r = (p0[v] + p1[v]) + (p2[v] + p3[v]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int idx = 4 * f + e;
            const int tap = idx / (C * C);
            const int rem = idx - tap * C * C;
            const int co = rem / C, ci = rem - co * C;
            dw[(co * C + ci) * 9 + tap] = r[e];
        }
    }
}

}  // namespace azg
