// Board-resident residual tower (split-fp16 products, C = 128): the eval forward's
// 2*NB residual convs (network.py:98-99, ResidualBlock network.py:9-26) with ONE board's
// activations held in LDS from the stem output to the tower output.
//
// Why: the tile towers (pv_tower.hip) re-stage every conv's halo from HBM / L2 (1.64x
// the algorithmic bytes at the self-play batch), pay an LDS round trip per operand
// (halo rows split to fp16 hi / lo while staged, weights through VGPRs and ds_write:
// ~0.9 LDS-array cycles per MFMA cycle) and hand tiles over between workgroups.  A
// 15x15 board with 128 channels is 115 KB as split fp16 -- it fits a CU's 160 KB LDS.
// One 16-wave workgroup per CU takes a board, converts its stem output to hi / lo once,
// and runs every conv from LDS: a conv's epilogue (BN, residual, ReLU) writes the next
// conv's operand straight back into LDS as hi / lo.  Only the block outputs go to HBM
// (in place over the stem output: each is the next block's fp32 residual and, for the
// last block, the heads' input).  Weights stream through two 16 KB LDS stages by LDS-DMA
// (one (tap, channel group) chunk per stage, one piece per wave), continuously across
// layers and boards.  No workgroup waits on another: there is no inter-workgroup
// hand-off at all.
//
// Work split: a board is 8 M fragments of 32 pixels (the last holds pixel 224 only: the
// 32x32 MFMA rows past 225 are padding) x 4 N fragments of 32 channels; wave w owns M
// fragment w % 8 and N fragments 2 (w / 8) .. +1 (a 32x64 wave tile: per K16 step 2 A and
// 4 B fragment reads for 6 MFMAs).
//
// Numerics: per output element the same MFMA sequence as halo_tile's split-fp16 body
// (pv_halo.h VAR bit 64) -- per channel group cg a chain over taps 0..8 and K16 steps
// (channels 16 st + 8 h + 0..7 of each lane) of lo_a hi_b, hi_a lo_b, hi_a hi_b into a
// zeroed accumulator, the group sums added in cg order, and the eval epilogue's explicit
// fmaf + residual + ReLU -- so the board tower is bitwise equal to the tile towers and
// the per-layer convs (tested), and the forward stays batch-independent.  A non-finite
// accumulator (an activation at or above 65520, beyond fp16) posts the launch to the H3
// overflow ring like every split-fp16 form; azg_pv_recover recomputes it in fp32.
#include "pv_internal.h"
#include "pv_halo.h"

namespace azg {

constexpr int kBtC = 128;
constexpr int kBtGroups = kBtC / 32;                         // channel groups
constexpr int kBtRows = PIX + 1;                             // 225 pixels + one zero row per group
constexpr int kBtStage = kBtC * 128;                         // one weight chunk: 128 rows x [hi 32 | lo 32] fp16
constexpr int kBtAct = 2 * kBtStage;                         // LDS: [2] weight stages, then the activations
constexpr int kBtProw = kBtAct + kBtGroups * kBtRows * 128;  // [4][226][128 B], then int prow[256]
constexpr int kBtLds = kBtProw + 256 * 4;                    // 149,504 B: one workgroup per CU
constexpr int kBtThreads = 1024;
constexpr int kBtMaxLayers = 2 * kTowerMaxBlocks;
constexpr int kBtStages = 9 * kBtGroups;                     // weight stages per conv

struct BoardArgs {
    const float* wp[kBtMaxLayers];      // split-fp16 packs of each conv (pack_h3: [tap*CG + cg][cout][hi 32 | lo 32])
    const float* scale[kBtMaxLayers];   // H3 BN scale (carries the pack's 2^-e) and shift
    const float* shift[kBtMaxLayers];
    float* x;                           // padded NHWC [B][17][17][128]: stem output in, tower output out
    int B;
    int nlayers;
    unsigned* ring_ovf;                 // host-mapped H3 overflow ring (device alias)
    unsigned seq;                       // launch number (0: autotuning runs, never posted)
};

__device__ __forceinline__ unsigned pack_f16x2(_Float16 a, _Float16 b)
{
    return (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
}

// Eval epilogue of one conv for a wave's 32x64 tile: y = relu(fmaf(acc, scale, shift)
// [+ the block input]) (halo_epilogue's arithmetic, element for element).  RES (conv2):
// the block input is read from and the block output written to the board's padded
// NHWC rows in HBM (in place; the same lane reads then writes each element).  y
// (TO_LDS) becomes the next conv's operand, [hi | lo] fp16 in the swizzled LDS rows: lane pairs
// (channels 2k, 2k + 1 of one pixel) exchange y by DPP and the even lane stores both hi
// halves, the odd lane both lo halves (one 4-B store each).  FULL: every row of the
// wave's M fragment is a pixel (M fragments 0..6; the 8th holds pixel 224 only), so no
// element is predicated.  Returns whether a valid accumulator was non-finite (an
// activation beyond fp16's range).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <bool RES, bool FULL, bool TO_LDS, int EABL = 0>
__device__ __forceinline__ bool bt_epilogue(const f32x16 (&acc)[2], const float* __restrict__ scale,
                                            const float* __restrict__ shift, float* __restrict__ xb, char* lds,
                                            const int* prow, int mf, int nh, int r32, int h)
{
    // element r of a fragment is pixel m = mf*32 + (r & 3) + 8 (r >> 2) + 4 h; its row key
    // (m >> 1) & 7 = 2 h ^ kr with kr = ((r >> 1) & 1) | (((r >> 2) & 1) << 2), so the store
    // slot is s1 ^ kr with the lane's s1 = (odd ? 4 : 0) + ((r32 & 30) >> 3) ^ 2 h: four
    // lane addresses (kr = 0, 1, 4, 5) and immediate offsets for the row and the N fragment
    int pr[16];
    if (RES || !FULL) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const int4 p4 = *(const int4*)(prow + mf * 32 + 8 * qd + 4 * h);
            pr[4 * qd] = p4.x, pr[4 * qd + 1] = p4.y, pr[4 * qd + 2] = p4.z, pr[4 * qd + 3] = p4.w;
        }
    }
    const int odd = r32 & 1, ce = r32 & 30;
    const int s1 = ((odd ? 4 : 0) + (ce >> 3)) ^ (2 * h);
    const int wbase = kBtAct + ((2 * nh) * kBtRows + mf * 32 + 4 * h) * 128 + (ce & 7) * 2;
    int wa[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wa[u] = wbase + 16 * (s1 ^ ((u & 1) | ((u >> 1) << 2)));
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = 64 * nh + 32 * j + r32;
        const float sj = scale[c], tj = shift[c];
        float rv[16];   // the block input of this N fragment, all loads in flight at once
        if constexpr (RES) {
#pragma unroll
            for (int r = 0; r < 16; ++r) rv[r] = (!(EABL & 8) && (FULL || pr[r] >= 0)) ? xb[pr[r] * kBtC + c] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = acc[j][r];
            const bool ok = FULL || pr[r] >= 0;
            bad |= ok && !__builtin_isfinite(v);
            const float y = RES ? fmaxf(fmaf(v, sj, tj) + rv[r], 0.f) : fmaxf(fmaf(v, sj, tj), 0.f);
            if (RES && ok && !(EABL & 8)) xb[pr[r] * kBtC + c] = y;
            if ((EABL & 8) && y == 1234.5f) xb[r] = y;
            if constexpr (TO_LDS) {
                const float yo =
                    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, y), 0xB1, 0xF, 0xF, false));
                const f32x2 yy = odd ? f32x2{yo, y} : f32x2{y, yo};
                const f16x2 hp = __builtin_convertvector(yy, f16x2);
                const f16x2 lp = __builtin_convertvector(yy - __builtin_convertvector(hp, f32x2), f16x2);
                const unsigned word = __builtin_bit_cast(unsigned, odd ? lp : hp);
                const int u = ((r >> 1) & 1) | (((r >> 2) & 1) << 1);
                const int off = j * kBtRows * 128 + ((r & 3) + 8 * (r >> 2)) * 128;
                if (ok && !(EABL & 16)) *(unsigned*)(lds + wa[u] + off) = word;
                if ((EABL & 16) && word == 12345u) xb[r] = y;
            }
        }
    }
    return bad;
}

int g_board_abl = 0;   // timing ablations of the board towers (key 51, study build): 1 no DMA wait, 2 no barrier, 4 no epilogue
template <int ABL>
__global__ __launch_bounds__(kBtThreads, 4) void board_tower(const BoardArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem_f[];
    char* lds = (char*)smem_f;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int mf = wid & 7, nh = wid >> 3;
    const int r32 = lane & 31, h = lane >> 5;
    int* prow = (int*)(lds + kBtProw);

    // padded row of every pixel (-1: the fragment padding past pixel 224), zero rows
    for (int i = tid; i < 256; i += kBtThreads) prow[i] = i < PIX ? (i / BOARD + 1) * PADW + i % BOARD + 1 : -1;
    if (tid < kBtGroups * 32) ((float*)(lds + kBtAct + ((tid >> 5) * kBtRows + PIX) * 128))[tid & 31] = 0.f;

    // this lane's A-fragment pixel and the taps that stay on the board
    int p = mf * 32 + r32;
    const int py = p / BOARD, px = p - py * BOARD;
    unsigned tmask = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
        if (p < PIX && yy >= 0 && yy < BOARD && xx >= 0 && xx < BOARD) tmask |= 1u << t;
    }
    // B fragments: weight row n = 64 nh + 32 j + r32 (key (n >> 1) & 7 = (r32 >> 1) & 7);
    // the slot of K16 step st (hi: c = 2 st + h, lo: 4 + 2 st + h) is c ^ key, so the
    // four reads of a lane are b0 ^ (32 m') with m' = st (hi) or 2 + st (lo)
    const int bkey = (r32 >> 1) & 7;
    const int b0 = (64 * nh + r32) * 128 + 32 * (bkey >> 1) + 16 * (h ^ (bkey & 1));

    // weight DMA: wave w moves rows 8 w .. 8 w + 7 of a chunk; lane -> row 8 w + lane / 8,
    // LDS slot lane % 8 holding source slot (lane % 8) ^ key(row)
    const int wrow = 8 * wid + (lane >> 3);
    const int wsrc = wrow * 32 + (((lane & 7) ^ ((wrow >> 1) & 7)) * 4);
    auto dma = [&](int l, int s, int buf) {
        const int cg = s / 9, tap = s - cg * 9;
        const float* src = a.wp[l] + (size_t)(tap * kBtGroups + cg) * kBtC * 32 + wsrc;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(lds + buf * kBtStage + wid * 1024),
                                         16, 0, 0);
    };

    const int nl = a.nlayers;
    int board = blockIdx.x;
    if (board < a.B) dma(0, 0, 0);
    __syncthreads();   // prow / zero rows
    for (; board < a.B; board += gridDim.x) {
        float* xb = a.x + (size_t)board * PADPIX * kBtC;
        int t8 = tid;
        asm volatile("" : "+v"(t8));   // the staging addresses are rebuilt per board, not kept live
        // ---- the board's stem output -> hi / lo rows [group][pixel] ----
        {
            f32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = t8 + k * kBtThreads;   // (pixel, float4 of 128 channels)
                if (i < PIX * 32) v[k] = *(const f32x4*)(xb + prow[i >> 5] * kBtC + (i & 31) * 4);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = t8 + k * kBtThreads;
                if (i < PIX * 32) {
                    const int m = i >> 5, c4 = i & 31, g = c4 >> 3, q4 = c4 & 7, key = (m >> 1) & 7;
                    f16x4 hi, lo;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        hi[e] = (_Float16)v[k][e];
                        lo[e] = (_Float16)(v[k][e] - (float)hi[e]);
                    }
                    char* row = lds + kBtAct + (g * kBtRows + m) * 128;
                    *(f16x4*)(row + (((q4 >> 1) ^ key) * 16) + (q4 & 1) * 8) = hi;
                    *(f16x4*)(row + (((4 + (q4 >> 1)) ^ key) * 16) + (q4 & 1) * 8) = lo;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's piece of the first stage
        __syncthreads();
        const bool more_boards = board + (int)gridDim.x < a.B;

        for (int l = 0; l < nl; ++l) {
            f32x16 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
            for (int cg = 0; cg < kBtGroups; ++cg) {
                f32x16 at[2];
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) at[j][r] = 0.f;
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    const int s = cg * 9 + tap;
                    const int buf = s & 1;
                    // the next stage's chunk into the other buffer (every wave is past its
                    // reads of that buffer: the barrier that ended the previous stage)
                    if (s + 1 < kBtStages) dma(l, s + 1, buf ^ 1);
                    else if (l + 1 < nl) dma(l + 1, 0, buf ^ 1);
                    else if (more_boards) dma(0, 0, buf ^ 1);
                    // the tap's A rows: neighbour pixel q (the group's zero row off the board)
                    // (rebuilt per tap: 36 hoisted row addresses would not fit the 128 VGPRs)
                    asm volatile("" : "+v"(tmask), "+v"(p));
                    const int d = (tap / 3 - 1) * BOARD + (tap % 3 - 1);
                    const int q = ((tmask >> tap) & 1) ? p + d : PIX;
                    const int k = (q >> 1) & 7;
                    const int a0 = kBtAct + (cg * kBtRows + q) * 128 + 32 * (k >> 1) + 16 * (h ^ (k & 1));
                    const char* bb = lds + buf * kBtStage;
#pragma unroll
                    for (int st = 0; st < 2; ++st) {
                        const f16x8 ah = *(const f16x8*)(lds + (a0 ^ (32 * st)));
                        const f16x8 al = *(const f16x8*)(lds + (a0 ^ (32 * (2 + st))));
                        f16x8 bh[2], bl[2];
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            bh[j] = *(const f16x8*)(bb + (b0 ^ (32 * st)) + j * 4096);
                            bl[j] = *(const f16x8*)(bb + (b0 ^ (32 * (2 + st))) + j * 4096);
                        }
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            at[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], at[j], 0, 0, 0);
                            at[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], at[j], 0, 0, 0);
                            at[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], at[j], 0, 0, 0);
                        }
                    }
                    // the next chunk has landed (this wave's piece) and every wave is past
                    // its reads of this stage's buffer
                    if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if constexpr (!(ABL & 2)) __syncthreads();
                    else __builtin_amdgcn_s_waitcnt(0xc07f);
                }
                // group boundary: fold this group's chain into acc HERE (the empty asm pins
                // the sum; left alone, LLVM sinks the four groups' adds to the end and keeps
                // every group's chain live: 128 spilled VGPRs)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[j] += at[j];
                    asm volatile("" : "+v"(acc[j]));
                }
            }

            // ---- epilogue: BN (+ block input) + ReLU; every wave is past its last read of
            // this conv's input (the barrier above) ----
            bool bad = false;
            if (ABL & 4) { if (acc[0][0] == 1234.5f) xb[tid] = acc[1][1]; }
            else {
                const float *sc = a.scale[l], *sh = a.shift[l];
#define AZG_BT_EPI(RES, FULL, TO) bad = bt_epilogue<RES, FULL, TO, ABL>(acc, sc, sh, xb, lds, prow, mf, nh, r32, h)
                if (mf < 7) {   // (wave-uniform)
                    if (!(l & 1)) AZG_BT_EPI(false, true, true);
                    else if (l + 1 < nl) AZG_BT_EPI(true, true, true);
                    else AZG_BT_EPI(true, true, false);
                } else {
                    if (!(l & 1)) AZG_BT_EPI(false, false, true);
                    else if (l + 1 < nl) AZG_BT_EPI(true, false, true);
                    else AZG_BT_EPI(true, false, false);
                }
#undef AZG_BT_EPI
            }
            if (bad && a.ring_ovf && a.seq)
                __hip_atomic_store(a.ring_ovf + (a.seq & (kH3RingSize - 1)), a.seq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            // the next conv reads what every wave wrote (and the next stage's chunk, issued at
            // the top of this conv's last stage, has landed: that stage's wait)
            __syncthreads();
        }
    }
}

hipError_t launch_board_tower(int NB, const float* wp16, const float* scale16, const float* shift, const int* out_off,
                              float* x, int B, unsigned* ring_ovf, unsigned seq, hipStream_t st)
{
    if (2 * NB > kBtMaxLayers || NB <= 0 || B <= 0) return hipErrorInvalidValue;
    static int grid = 0;
    if (grid == 0) {
        hipError_t e = hipSuccess;
#ifdef AZG_AB_STUDIES
        for (const void* f : {(const void*)board_tower<0>, (const void*)board_tower<1>, (const void*)board_tower<2>,
                              (const void*)board_tower<4>, (const void*)board_tower<7>, (const void*)board_tower<8>,
                              (const void*)board_tower<16>, (const void*)board_tower<24>})
#else
        for (const void* f : {(const void*)board_tower<0>})
#endif
            if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kBtLds)) != hipSuccess) return e;
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)board_tower<0>, kBtThreads, kBtLds);
        if (e != hipSuccess) return e;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        if (per_cu < 1) return hipErrorInvalidConfiguration;
        grid = per_cu * cus;
    }
    BoardArgs a{};
    for (int l = 0; l < 2 * NB; ++l) {
        a.wp[l] = wp16 + (size_t)l * 9 * kBtC * kBtC;
        a.scale[l] = scale16 + out_off[l];
        a.shift[l] = shift + out_off[l];
    }
    a.x = x;
    a.B = B;
    a.nlayers = 2 * NB;
    a.ring_ovf = ring_ovf;
    a.seq = seq;
    const dim3 g(B < grid ? B : grid);
#ifdef AZG_AB_STUDIES
    switch (g_board_abl) {   // timing ablations (key 51, study build; results invalid while set)
        case 1: hipLaunchKernelGGL(board_tower<1>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 2: hipLaunchKernelGGL(board_tower<2>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 4: hipLaunchKernelGGL(board_tower<4>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 7: hipLaunchKernelGGL(board_tower<7>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 8: hipLaunchKernelGGL(board_tower<8>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 16: hipLaunchKernelGGL(board_tower<16>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        case 24: hipLaunchKernelGGL(board_tower<24>, g, dim3(kBtThreads), kBtLds, st, a); return hipGetLastError();
        default: break;
    }
#endif
    hipLaunchKernelGGL(board_tower<0>, g, dim3(kBtThreads), kBtLds, st, a);
    return hipGetLastError();
}

}  // namespace azg
