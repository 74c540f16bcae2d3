// Weight gradient of the 3x3 convolution (autograd of network.py:12,14 conv2d):
//   dW[co][ci][tap] = sum_m dz[m][co] * X[m + off(tap)][ci]
// as an fp32-MFMA GEMM with co x ci outputs per tap and K = pixels of the batch,
// split over pixel slabs (split-K) so the grid fills the chip: every workgroup
// writes its 128x128 (64x64 at C=64) partial tile to a slab; wgrad_reduce sums
// the slabs in a fixed order (bitwise reproducible) into torch's [Cout][Cin][3][3].
//
// Split s covers the whole 32-pixel chunks [s*NCH/S, (s+1)*NCH/S) of the batch
// (NCH = ceil(M/32)): every split has 16 or 17 chunks at B = 128 instead of a fixed
// row count whose last chunk is mostly padding.  Rows past M load zeros.
#include "pv_internal.h"

namespace azg {

__device__ __forceinline__ void wgrad_split_rows(int split, int S, int M, int& mbeg, int& mend)
{
    const int nch = (M + 31) / 32;
    mbeg = (int)((int64_t)split * nch / S) * 32;
    mend = min(M, (int)((int64_t)(split + 1) * nch / S) * 32);
}

template <int C, int BK_ = 32>
struct WgTile {
    static constexpr int BT = C < 128 ? C : 128;    // tile edge (co and ci)
    static constexpr int BK = BK_;                  // pixels per chunk
    static constexpr int LD = BT + 4;
    static constexpr int W = BT / 2;                // per-wave edge (2x2 waves)
    static constexpr int T = W / 32;                // 32x32 MFMA tiles per wave edge
    static constexpr int LDF4 = BK * BT / 4 / 256;  // float4 per thread per operand
    static constexpr int NT = C / BT;               // tiles per edge
    static constexpr int LDS_BYTES = 2 * 2 * BK * LD * 4;
};

template <int C, int BK_ = 32>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_mfma(
    const float* __restrict__ dz,   // padded NHWC [B][17][17][C]  (A^T: co)
    const float* __restrict__ x,    // padded NHWC                 (B: ci)
    float* __restrict__ slab,       // [S][9][C][C] partial dW[tap][co][ci]
    int M, int S)
{
    using T = WgTile<C, BK_>;
    constexpr int BT = T::BT, BK = T::BK, LD = T::LD, W = T::W, TT = T::T, LDF4 = T::LDF4, NT = T::NT;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                 // [2][BK][LD]  dz rows
    float* Bs = smem + 2 * BK * LD;   // [2][BK][LD]  x rows

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    // XCD-aware order (cdna_hip_programming.md T1; speed only): blocks b and b+8
    // share an XCD, so every tile of one pixel split is given to the same block
    // label b % 8 -- the split's dz rows and (tap-shifted) x rows are fetched into
    // that XCD's L2 once and served to all 9*NT*NT of its tiles.  gridDim.x =
    // S * tiles with S % 8 == 0.
    constexpr int TILES = 9 * NT * NT;
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int split = (k / TILES) * 8 + xcd;
    int t = k % TILES;
    const int tap = t / (NT * NT);
    t -= tap * NT * NT;
    const int co0 = (t / NT) * BT, ci0 = (t % NT) * BT;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    int mbeg, mend;
    wgrad_split_rows(split, S, M, mbeg, mend);
    const int nch = (mend - mbeg + BK - 1) / BK;

    // staging: LDF4 float4 per thread per operand; thread -> (row, col4)
    constexpr int F4_PER_ROW = BT / 4;
    f32x4 ra[LDF4], rb[LDF4];
    auto gload = [&](int kc) {
#pragma unroll
        for (int i = 0; i < LDF4; ++i) {
            const int f = tid + 256 * i;
            const int r = f / F4_PER_ROW, c4 = (f - r * F4_PER_ROW) * 4;
            const int m = mbeg + kc * BK + r;
            if (m < mend) {
                const int po = pad_off(m, C);
                ra[i] = *(const f32x4*)(dz + po + co0 + c4);
                rb[i] = *(const f32x4*)(x + po + toff + ci0 + c4);
            } else {
                ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < LDF4; ++i) {
            const int f = tid + 256 * i;
            const int r = f / F4_PER_ROW, c4 = (f - r * F4_PER_ROW) * 4;
            *(f32x4*)(As + buf * BK * LD + r * LD + c4) = ra[i];
            *(f32x4*)(Bs + buf * BK * LD + r * LD + c4) = rb[i];
        }
    };

    f32x16 acc[TT][TT];
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int r32 = lane & 31, h = lane >> 5;
    if (nch > 0) {
        gload(0);
        lstore(0);
    }
    __syncthreads();
    for (int kc = 0; kc < nch; ++kc) {
        const int cur = kc & 1;
        if (kc + 1 < nch) gload(kc + 1);
        // keep the next chunk's global loads at the top of the chunk: without this
        // fence hipcc sinks them to just before their vmcnt wait (latency exposed)
        __builtin_amdgcn_sched_barrier(0);
        const float* Ab = As + cur * BK * LD + (h * (BK / 2)) * LD + wm * W + r32;
        const float* Bb = Bs + cur * BK * LD + (h * (BK / 2)) * LD + wn * W + r32;
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float a[TT], b[TT];
#pragma unroll
            for (int i = 0; i < TT; ++i) a[i] = Ab[s * LD + i * 32];
#pragma unroll
            for (int j = 0; j < TT; ++j) b[j] = Bb[s * LD + j * 32];
#pragma unroll
            for (int i = 0; i < TT; ++i)
#pragma unroll
                for (int j = 0; j < TT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (kc + 1 < nch) lstore(cur ^ 1);
        __syncthreads();
    }

    // D[i = co][j = ci]: col = lane&31 (ci), row = (r&3) + 8*(r>>2) + 4*h (co)
    float* out = slab + ((size_t)split * 9 + tap) * C * C;
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm * W + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int ci = ci0 + wn * W + j * 32 + r32;
                out[co * C + ci] = acc[i][j][r];
            }
}

// Same GEMM with K-CONTIGUOUS operand staging: each thread loads a 4-pixel x
// 4-channel block of dz and of the tap-shifted x (four 16-B loads), transposes it
// in registers and writes four 16-B channel rows [c][pix] to LDS, so the MFMA
// fragments (lane = one co / ci, 4 consecutive pixels of its K half) are 16-B
// ds_read_b128 instead of one ds_read_b32 per MFMA: per 32-pixel chunk a wave
// issues 16 fragment reads for its 64 MFMAs (was 64).  K order per output: chunks
// in order, within a chunk pixel pairs (s, 16+s), s = 0..15.
// PF2: global loads issued two chunks ahead (two register sets, the loop unrolled
// by two so the sets are static): a load has a whole chunk of MFMAs more to land.
template <int C, bool PF2 = false, bool WT = false>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_t(
    const float* __restrict__ dz, const float* __restrict__ x, float* __restrict__ slab, int M, int S)
{
    using T = WgTile<C, 32>;
    constexpr int BT = T::BT, BK = 32, W = T::W, TT = T::T, NT = T::NT;
    constexpr int LDT = BK + 4;                       // 36: conflict-free b128 reads, 16-B aligned rows
    constexpr int NBLK = (BT / 4) * (BK / 4);         // 4x4 staging blocks per operand per chunk
    static_assert(NBLK <= 256, "one staging block per thread");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                                 // [2][BT][LDT] dz^T
    float* Bs = smem + 2 * BT * LDT;                  // [2][BT][LDT] x^T (tap-shifted)

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    constexpr int TILES = 9 * NT * NT;
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;   // XCD-aware order, see conv3x3_wgrad_mfma
    const int split = (k / TILES) * 8 + xcd;
    int t = k % TILES;
    const int tap = t / (NT * NT);
    t -= tap * NT * NT;
    const int co0 = (t / NT) * BT, ci0 = (t % NT) * BT;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    int mbeg, mend;
    wgrad_split_rows(split, S, M, mbeg, mend);
    const int nch = (mend - mbeg + BK - 1) / BK;

    const bool stager = tid < NBLK;
    const int pb = tid % (BK / 4), cb = tid / (BK / 4);     // pixel block, channel block
    f32x4 ra[4], rb[4], ra2[4], rb2[4];
    auto gload_to = [&](int kc, f32x4 (&xa)[4], f32x4 (&xb)[4]) {
        if (!stager) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mbeg + kc * BK + 4 * pb + i;
            if (m < mend) {
                const int po = pad_off(m, C);
                xa[i] = *(const f32x4*)(dz + po + co0 + 4 * cb);
                xb[i] = *(const f32x4*)(x + po + toff + ci0 + 4 * cb);
            } else {
                xa[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                xb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto lstore_from = [&](int buf, const f32x4 (&xa)[4], const f32x4 (&xb)[4]) {
        if (!stager) return;
        float* a = As + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
        float* b = Bs + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            *(f32x4*)(a + j * LDT) = f32x4{xa[0][j], xa[1][j], xa[2][j], xa[3][j]};
            *(f32x4*)(b + j * LDT) = f32x4{xb[0][j], xb[1][j], xb[2][j], xb[3][j]};
        }
    };
    auto gload = [&](int kc) {
        if (!stager) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mbeg + kc * BK + 4 * pb + i;
            if (m < mend) {
                const int po = pad_off(m, C);
                ra[i] = *(const f32x4*)(dz + po + co0 + 4 * cb);
                rb[i] = *(const f32x4*)(x + po + toff + ci0 + 4 * cb);
            } else {
                ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto lstore = [&](int buf) {
        if (!stager) return;
        float* a = As + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
        float* b = Bs + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            *(f32x4*)(a + j * LDT) = f32x4{ra[0][j], ra[1][j], ra[2][j], ra[3][j]};
            *(f32x4*)(b + j * LDT) = f32x4{rb[0][j], rb[1][j], rb[2][j], rb[3][j]};
        }
    };

    f32x16 acc[TT][TT];
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int r32 = lane & 31, h = lane >> 5;
    auto compute = [&](int cur) {
        const float* Ab = As + cur * BT * LDT + (wm * W + r32) * LDT + h * (BK / 2);
        const float* Bb = Bs + cur * BT * LDT + (wn * W + r32) * LDT + h * (BK / 2);
#pragma unroll
        for (int q = 0; q < BK / 8; ++q) {
            f32x4 a[TT], b[TT];
#pragma unroll
            for (int i = 0; i < TT; ++i) a[i] = *(const f32x4*)(Ab + i * 32 * LDT + 4 * q);
#pragma unroll
            for (int j = 0; j < TT; ++j) b[j] = *(const f32x4*)(Bb + j * 32 * LDT + 4 * q);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                for (int i = 0; i < TT; ++i)
#pragma unroll
                    for (int j = 0; j < TT; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s4], b[j][s4], acc[i][j], 0, 0, 0);
        }
    };
    if constexpr (PF2) {
        // chunk j lives in register set j & 1 from its load (two chunks ahead) to its
        // LDS store (end of chunk j - 1)
        if (nch > 0) {
            gload_to(0, ra, rb);
            lstore_from(0, ra, rb);
        }
        if (nch > 1) gload_to(1, ra2, rb2);
        __syncthreads();
        auto iter = [&](int kc, f32x4 (&la)[4], f32x4 (&lb)[4], f32x4 (&sa)[4], f32x4 (&sb)[4]) {
            if (kc + 2 < nch) gload_to(kc + 2, la, lb);
            __builtin_amdgcn_sched_barrier(0);
            compute(kc & 1);
            if (kc + 1 < nch) lstore_from((kc + 1) & 1, sa, sb);
            __syncthreads();
        };
        for (int kc = 0; kc < nch; kc += 2) {
            iter(kc, ra, rb, ra2, rb2);
            if (kc + 1 < nch) iter(kc + 1, ra2, rb2, ra, rb);
        }
    } else {
        if (nch > 0) {
            gload(0);
            lstore(0);
        }
        __syncthreads();
        for (int kc = 0; kc < nch; ++kc) {
            const int cur = kc & 1;
            if (kc + 1 < nch) gload(kc + 1);
            __builtin_amdgcn_sched_barrier(0);
            compute(cur);
            if (kc + 1 < nch) lstore(cur ^ 1);
            __syncthreads();
        }
    }

    float* out = slab + ((size_t)split * 9 + tap) * C * C;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, (size_t)C * C * sizeof(float));
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm * W + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int ci = ci0 + wn * W + j * 32 + r32;
                store1<WT>(out, rs, co * C + ci, acc[i][j][r]);
            }
}


// Same GEMM with NATURAL operand rows in LDS filled by LDS-DMA (default, key 16 = 3):
// each wave-instruction global_load_lds_dwordx4 moves 1 KiB = 256/BT pixel rows of
// BT channels straight into LDS (no staging VGPRs, no register transposition, no
// ds_write), issued one chunk ahead.  MFMA step s reads, per operand, one
// ds_read_b32 per lane: lanes 0-31 pixel s, lanes 32-63 pixel s + 16, 32
// consecutive channels (co for dz, ci for x) -- the same K order as
// conv3x3_wgrad_t, so all three kernels are bitwise identical.  16-B chunk j of LDS
// row p holds global chunk j ^ 8*((p >> 4) & 1) (swizzle applied to each lane's
// source address, cdna_hip_programming.md §5.4): the two half-waves of a fragment
// read land on disjoint bank halves.  Rows past the split read padded pixel 0 (the
// zero halo).  Measured at 6x128, B = 128 (scripts/wgrad_lab.hip): 74.0 vs 89.2 us
// (hipEvent incl. launch) for the K-contiguous kernel.
// COMB (key 41, with WT): the S/8 splits of one pixel-split group (splits g, g + 8, ...:
// the XCD-aware order puts them on one XCD) combine in-kernel -- every workgroup stores
// its slab write-through, drains, meets a barrier and counts the tile on the group's
// agent-scope counter (R1); the workgroup whose add returns the last count runs ONE
// agent-scope acquire + vmcnt(0), then sums the group's slabs of its tile in split
// order (plain loads) into the group slab gslab[g] (write-through).  wgrad_reduce then
// reads 8 group slabs instead of S: 4.7 instead of 33 MB per conv at 6x128, B = 128.
template <int C, bool WT = true, int NWV = 4, bool COMB = false>
__global__ __launch_bounds__(64 * NWV, 2) void conv3x3_wgrad_nat(
    const float* __restrict__ dz, const float* __restrict__ x, float* __restrict__ slab, int M, int S,
    unsigned* __restrict__ gcnt = nullptr, float* __restrict__ gslab = nullptr)
{
    // NWV = 4: 2 x 2 waves of (BT/2) x (BT/2); NWV = 8 (BT = 128): 2 x 4 waves of 64 co x
    // 32 ci (two accumulators each: four waves per SIMD at two workgroups per CU;
    // measured equal to NWV = 4)
    constexpr int BT = C < 128 ? C : 128, BK = 32, NT = C / BT;
    constexpr int WNW = NWV == 8 ? 4 : 2;           // waves along ci
    constexpr int TA = BT / 64, TB = BT / (32 * WNW); // accumulators along co / ci per wave
    constexpr int RPI = 256 / BT;      // pixel rows per wave-instruction (1 KiB)
    constexpr int CPR = BT / 4;        // 16-B chunks per row
    constexpr int IPW = BK / RPI / NWV;  // instructions per wave per operand per chunk
    static_assert(IPW >= 1 && CPR >= 16 && TB >= 1, "tile");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                  // [2][BK][BT]  dz rows (co)
    float* Bs = smem + 2 * BK * BT;    // [2][BK][BT]  x rows (ci, tap-shifted)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WNW, wn = wid % WNW;
    constexpr int TILES = 9 * NT * NT;
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;   // XCD-aware order, see conv3x3_wgrad_mfma
    const int split = (k / TILES) * 8 + xcd;
    int t = k % TILES;
    const int tap = t / (NT * NT);
    t -= tap * NT * NT;
    const int co0 = (t / NT) * BT, ci0 = (t % NT) * BT;
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
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of chunk kc+1 retired
        __syncthreads();
    }

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
    if constexpr (COMB) {
        static_assert(WT, "the group combine reads slabs stored write-through");
        __shared__ unsigned flag;
        const int tid_ = threadIdx.x;
        const int g = xcd, tileid = k % TILES, nmem = S / 8;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid_ == 0) {
            unsigned* c = gcnt + tileid * 8 + g;
            const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned last = old == (unsigned)(nmem - 1) ? 1u : 0u;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-armed
            }
            flag = last;
        }
        __syncthreads();
        if (flag) {
            // this tile's BT x BT region of tap `tap`: float4 runs, the group's slabs in
            // split order, every load of a run issued before its sum
            constexpr int NTH = 64 * NWV, F4 = BT * BT / 4 / NTH, MMAX = 8;
            float* gout = gslab + ((size_t)g * 9 + tap) * C * C;
            const __amdgpu_buffer_rsrc_t grs = wt_rsrc(gout, (size_t)C * C * sizeof(float));
            for (int u = 0; u < F4; ++u) {
                const int e = (tid_ + NTH * u) * 4;
                const size_t off = (size_t)(co0 + e / BT) * C + ci0 + e % BT;
                f32x4 sum = {0.f, 0.f, 0.f, 0.f};
                for (int m0 = 0; m0 < nmem; m0 += MMAX) {
                    f32x4 v[MMAX];
#pragma unroll
                    for (int m = 0; m < MMAX; ++m)
                        if (m0 + m < nmem)
                            v[m] = *(const f32x4*)(slab + ((size_t)((m0 + m) * 8 + g) * 9 + tap) * C * C + off);
#pragma unroll
                    for (int m = 0; m < MMAX; ++m)
                        if (m0 + m < nmem) sum += v[m];
                }
                store4<true>(gout, grs, (int)off, sum);
            }
        }
    }
}

// dW (torch layout [co][ci][3][3]) = sum over slabs, fixed order: four interleaved
// partial sums (slabs k = 0,1,2,3 mod 4: independent loads in flight) combined as
// ((p0 + p1) + (p2 + p3)).
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ slab, float* __restrict__ dw, int C, int S)
{
    const int total = 9 * C * C;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        // idx enumerates slab layout [tap][co][ci] (coalesced reads)
        const int tap = idx / (C * C);
        const int rem = idx - tap * C * C;
        const int co = rem / C, ci = rem - co * C;
        float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
        int k = 0;
        for (; k + 4 <= S; k += 4) {
            p0 += slab[(size_t)k * total + idx];
            p1 += slab[(size_t)(k + 1) * total + idx];
            p2 += slab[(size_t)(k + 2) * total + idx];
            p3 += slab[(size_t)(k + 3) * total + idx];
        }
        if (k < S) p0 += slab[(size_t)k * total + idx];
        if (k + 1 < S) p1 += slab[(size_t)(k + 1) * total + idx];
        if (k + 2 < S) p2 += slab[(size_t)(k + 2) * total + idx];
        dw[(co * C + ci) * 9 + tap] = (p0 + p1) + (p2 + p3);
    }
}
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                           int C, int S)
{
    wgrad_reduce_body(slab, dw, C, S);
}
// two convs' reductions in one launch (grid.y selects the conv; the same per-element
// order as wgrad_reduce_kernel, so bitwise identical to two launches)
__global__ __launch_bounds__(256) void wgrad_reduce2_kernel(const float* __restrict__ slab0, float* __restrict__ dw0,
                                                            int S0, const float* __restrict__ slab1,
                                                            float* __restrict__ dw1, int S1, int C)
{
    if (blockIdx.y == 0) wgrad_reduce_body(slab0, dw0, C, S0);
    else wgrad_reduce_body(slab1, dw1, C, S1);
}

// dW = the S slabs summed in fixed order (wgrad_reduce_kernel)
hipError_t launch_wgrad_reduce(int C, const float* slab, float* dw, int S, hipStream_t st)
{
    const int total = 9 * C * C;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, slab, dw, C, S);
    return hipGetLastError();
}

hipError_t launch_wgrad_reduce2(int C, const float* slab0, float* dw0, int S0, const float* slab1, float* dw1,
                                int S1, hipStream_t st)
{
    const int total = 9 * C * C;
    hipLaunchKernelGGL(wgrad_reduce2_kernel, dim3((total + 255) / 256, 2), dim3(256), 0, st, slab0, dw0, S0, slab1,
                       dw1, S1, C);
    return hipGetLastError();
}

// 3: LDS-DMA natural rows (conv3x3_wgrad_nat, default); 1: K-contiguous register
// staging; 2: the same two chunks ahead; 0: row staging (A/B; all bitwise identical)
int g_wgrad_kernel = 3;

bool wgrad_comb_on(int kernel, int S);
int g_wgrad_comb = 0;   // key 41: 1 in-kernel split-group combine of the LDS-DMA weight grad (slower, measured); 0 off (default)

template <int C, int BK = 32>
static hipError_t launch_wgrad_t(const float* dz, const float* x, float* slab, float* dw, int M, int S,
                                 hipStream_t st, bool reduce, unsigned* gcnt, float* gslab)
{
    using T = WgTile<C, BK>;
    if (S % 8) return hipErrorInvalidValue;           // wgrad_splits guarantees S % 8 == 0
    dim3 grid(S * 9 * T::NT * T::NT);
    if (g_wgrad_kernel >= 3 && BK == 32) {
        constexpr int lds = 2 * 2 * 32 * T::BT * 4;
        static bool attr_n = false;
        if (!attr_n) {
            hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat<C, true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat<C, false>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if constexpr (T::BT == 128)
                if (e == hipSuccess)
                    e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat<C, true, 8>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e != hipSuccess) return e;
            attr_n = true;
        }
        if constexpr (T::BT == 128) {
            if (g_wgrad_kernel == 4 && (g_train_wt & 4)) {   // 8 waves per 128x128 tile
                hipLaunchKernelGGL((conv3x3_wgrad_nat<C, true, 8>), grid, dim3(512), lds, st, dz, x, slab, M, S);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess || !reduce) return e;
                return launch_wgrad_reduce(C, slab, dw, S, st);
            }
        }
        if (wgrad_comb_on(g_wgrad_kernel, S) && gcnt && gslab) {
            static bool attr_c = false;
            if (!attr_c) {
                hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat<C, true, 4, true>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                if (e != hipSuccess) return e;
                attr_c = true;
            }
            hipLaunchKernelGGL((conv3x3_wgrad_nat<C, true, 4, true>), grid, dim3(256), lds, st, dz, x, slab, M, S, gcnt,
                               gslab);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess || !reduce) return e;
            return launch_wgrad_reduce(C, gslab, dw, 8, st);
        }
        if (g_train_wt & 4)
            hipLaunchKernelGGL((conv3x3_wgrad_nat<C, true>), grid, dim3(256), lds, st, dz, x, slab, M, S);
        else
            hipLaunchKernelGGL((conv3x3_wgrad_nat<C, false>), grid, dim3(256), lds, st, dz, x, slab, M, S);
    } else if (g_wgrad_kernel >= 1 && BK == 32) {
        constexpr int lds = 2 * 2 * T::BT * (32 + 4) * 4;
        static bool attr_t = false;
        if (!attr_t) {
            hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_t<C>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)conv3x3_wgrad_t<C, true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)conv3x3_wgrad_t<C, false, true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e != hipSuccess) return e;
            attr_t = true;
        }
        if (g_wgrad_kernel == 2)
            hipLaunchKernelGGL((conv3x3_wgrad_t<C, true>), grid, dim3(256), lds, st, dz, x, slab, M, S);
        else if (g_train_wt & 4)
            hipLaunchKernelGGL((conv3x3_wgrad_t<C, false, true>), grid, dim3(256), lds, st, dz, x, slab, M, S);
        else
            hipLaunchKernelGGL((conv3x3_wgrad_t<C>), grid, dim3(256), lds, st, dz, x, slab, M, S);
    } else {
        static bool attr_done = false;
        if (!attr_done) {
            hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_mfma<C, BK>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS_BYTES);
            if (e != hipSuccess) return e;
            attr_done = true;
        }
        hipLaunchKernelGGL((conv3x3_wgrad_mfma<C, BK>), grid, dim3(256), T::LDS_BYTES, st, dz, x, slab, M, S);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !reduce) return e;
    return launch_wgrad_reduce(C, slab, dw, S, st);
}

// Pixel splits: S is a multiple of 8 (the XCD-aware order keeps each split on one
// XCD); the smallest S whose S * tiles workgroups fill the resident slots in ONE
// round (fewest chunks per workgroup), falling back to whole rounds for tiny M;
// every split keeps >= 2 whole 32-pixel chunks.
int g_wgrad_bk = 32;   // pixels per K chunk of the row-staging tile (32 default; 16 = A/B study)

int g_wgrad_splits = 0;   // key 27: split-K count override (multiple of 8, <= 64; 0 = automatic)

int wgrad_splits(int C, int M)
{
    if (g_wgrad_splits > 0) {
        int S = g_wgrad_splits;
        const int nch = (M + 31) / 32;
        while (S > 8 && nch < 2 * S) S -= 8;
        return S;
    }
    const int bt = C < 128 ? C : 128;
    const int tiles = 9 * (C / bt) * (C / bt);
    const int lds = 2 * 2 * bt * (g_wgrad_bk + 4) * 4;   // largest variant (K-contiguous staging)
    const int per_cu = 160 * 1024 / lds < 2 ? 160 * 1024 / lds : 2;
    const int slots = 256 * per_cu;
    int S = (slots / tiles) / 8 * 8;
    if (S < 8) S = 8;
    const int nch = (M + 31) / 32;
    while (S > 8 && nch < 2 * S) S -= 8;
    return S;
}

// slab must hold S*9*C*C floats, S = wgrad_splits(C, M).
// the weight grad reduces S / 8 group slabs in-kernel (key 41): the LDS-DMA kernel
// (key 16 = 3) with write-through slabs
bool wgrad_comb_on(int kernel, int S)
{
    return g_wgrad_comb && kernel == 3 && (g_train_wt & 4) && S % 8 == 0 && g_wgrad_bk == 32;
}

hipError_t launch_wgrad(int C, const float* dz, const float* x, float* slab, float* dw, int M, int S,
                        hipStream_t st, bool reduce, unsigned* gcnt, float* gslab)
{
    switch (C) {
        case 64: return launch_wgrad_t<64>(dz, x, slab, dw, M, S, st, reduce, gcnt, gslab);
        case 128:
            if (g_wgrad_bk == 16) return launch_wgrad_t<128, 16>(dz, x, slab, dw, M, S, st, reduce, gcnt, gslab);
            return launch_wgrad_t<128>(dz, x, slab, dw, M, S, st, reduce, gcnt, gslab);
        case 256: return launch_wgrad_t<256>(dz, x, slab, dw, M, S, st, reduce, gcnt, gslab);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace azg
