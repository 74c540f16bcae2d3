// Board-resident residual tower on 16x16x32 products (split fp16, C = 128): the eval
// forward's 2*NB residual convs (network.py:98-99, ResidualBlock network.py:9-26), one
// board per 12-wave workgroup with the board's activations in LDS from the stem output to
// the tower output -- pv_board.hip's structure on v_mfma_f32_16x16x32_f16.
//
// Why a second board tower: on gfx950 a CU streaming 16x16x32 f16 MFMAs sustains ~1.2x the
// FLOP/s of one streaming 32x32x16 (scripts/lab/mfma_clock.hip: 2.05 vs 1.69 PFLOP/s
// chip-wide, the same instruction peak -- the clock the power limit allows), and 16-row
// fragments pad a board's 225 pixels to 240 rows instead of 256.  A 16x16x32 product sums
// 32 channels per instruction, so this tower is its own arithmetic class (key 19 = 2):
// within it every batch and every board computes the same MFMA sequence per element
// (batch-independent, as the K16 forms are among themselves), and it matches the fp32
// oracle to the split-fp16 tolerance.
//
// Work split: 15 M fragments of 16 pixels (the last holds pixel 224 only) x 8 N fragments
// of 16 channels; wave w owns M fragments 5 (w % 3) .. +4 and the output channel group
// w / 3 (32 channels: 2 N fragments) -- an 80x32 wave tile, per K32 step 10 A and 4 B
// fragment reads for 30 MFMAs.
//
// Numerics: per output element one chain over channel groups cg, taps 0..8 and the three
// products lo_a hi_b, hi_a lo_b, hi_a hi_b (channels 32 cg + 8 (lane >> 4) + 0..7 of each
// lane, the pack_h3 order), then the eval epilogue relu(fmaf(acc, scale, shift) [+ the
// block input]).  A non-finite accumulator (an activation at or above 65520) posts the
// launch to the H3 overflow ring; azg_pv_recover recomputes it in fp32.
//
// LDS rows: per channel group a [226][128 B] image (pixels 0..224, then a zero row: the
// neighbour of an off-board tap); a row's 16-B slots are {hi c 0-7, 8-15, 16-23, 24-31, lo
// ...} stored at slot ^ (row & 6).  That key keeps every ds_read_b128 of an A fragment
// conflict-free for every tap shift (a 16-lane bank group reads rows b + {0-3, 12-15} at
// slot k and b + {4-11} at slot k ^ 1, for any b), the B reads (weight rows, b = 0) and the
// epilogue's 4-B stores too.
#include "pv_internal.h"

namespace azg {

constexpr int kB16C = 128;
constexpr int kB16Groups = kB16C / 32;
constexpr int kB16Rows = PIX + 1;                             // 225 pixels + the zero row
constexpr int kB16Stage = kB16C * 128;                        // one (tap, cg) weight chunk: 128 rows x [hi 32 | lo 32]
constexpr int kB16Act = 2 * kB16Stage;                        // LDS: [2] weight stages, then the activations
constexpr int kB16Prow = kB16Act + kB16Groups * kB16Rows * 128;
constexpr int kB16Hw = kB16Prow + 240 * 4;                    // the heads' 1x1 weights [3][128] (fused projection)
constexpr int kB16Lds = kB16Hw + 3 * kB16C * 4;               // 150,976 B: one workgroup per CU
constexpr int kB16Waves = 12;
constexpr int kB16Threads = 64 * kB16Waves;
constexpr int kB16SplitThreads = 512;                         // SPLIT: 8 waves (80x16 tiles), one pixel third of a board
constexpr int kB16Img = kB16Groups * kB16Rows * 128;          // one board's image (an exchange buffer)
static_assert(kB16Img == (int)kB16ImgBytes, "pv_internal.h kB16ImgBytes");
constexpr int kB16MaxLayers = 2 * kTowerMaxBlocks;
constexpr int kB16Steps = 9 * kB16Groups;                     // K32 steps (weight chunks) per conv
static_assert((kB16Groups * kB16Rows * 128) % 256 == 0, "a group's image keeps the 256-B bank phase");
static_assert(kB16Steps % 2 == 0, "step s of every conv uses stage s & 1");

struct Board16Args {
    const float* wp[kB16MaxLayers];     // split-fp16 packs (pack_h3: [tap*CG + cg][cout][hi 32 | lo 32])
    const float* scale[kB16MaxLayers];  // H3 BN scale (carries the pack's 2^-e) and shift
    const float* shift[kB16MaxLayers];
    float* x;                           // padded NHWC [B][17][17][128]: stem output in, tower output out
    int B;
    int nlayers;
    unsigned* ring_ovf;                 // host-mapped H3 overflow ring (device alias)
    unsigned seq;                       // launch number (0: autotuning runs, never posted)
    const float* hwp;                   // heads: policy_conv [2][128], value_conv [128] weights,
    const float* hwv;                   //   folded BN scale / shift [3] (policy 2, value 1)
    const float* hsc;
    const float* hsh;
    float* hout;                        // [B][FC_FS] projected features (nullptr: tower output to x)
    // SPLIT (small batches): three workgroups per board exchange conv outputs' boundary rows
    char* xbuf;                         // [B][2 (layer parity)][kB16Img] exchange images
    unsigned* xflag;                    // [B][3] per pixel third: epoch * 64 + layers published
    unsigned epoch;                     // this launch's tag base (the handle's split launch count)
    unsigned* ring;                     // host-mapped ring of timed-out launches (azg_pv_recover)
    unsigned* diag;                     // the tower wait record (word 1: timeouts); may be null
    unsigned limit;                     // awake-time bound of one wait, 10-ns ticks (key 14)
};

typedef float b16_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned b16_u32x4 __attribute__((ext_vector_type(4)));

// byte offset of (pixel m, channel c) in the fp32 rows of the fused heads projection: 16-B
// slots keyed by m & 15, so the epilogue's stores and the projection's float4 reads spread
// over the banks (a wave's 16 pixels x 4 quarters read 64 distinct slots of 16 bank groups)
__device__ __forceinline__ int b16_f32_row(int m, int c) { return m * (kB16C * 4) + 16 * ((c >> 2) ^ (m & 15)) + 4 * (c & 3); }
typedef _Float16 b16_f16x2 __attribute__((ext_vector_type(2)));

// Eval epilogue of one conv for a wave's 80x32 tile: element i of tile (f, n) is pixel
// 80 mg + 16 f + 4 kb + i, channel 32 cg + 16 n + r16.  RES (conv2): the block input is
// read from and the block output written to the board's padded NHWC rows in HBM (in place,
// the same lane reads then writes each element) through a buffer resource: a padding
// pixel's row offset lies past the resource, so its load returns 0 and its store is
// dropped (no branches).  TO_LDS: y becomes the next conv's operand, [hi | lo] fp16 in the
// keyed rows: a lane splits its two elements (i, i + 1) together, H = (hi_i, hi_i+1) and L =
// (lo_i, lo_i+1); lane pairs (channels 2k, 2k + 1 of one pixel) hand over their H (to the
// even lane) or L (to the odd lane) by one DPP, and two v_perm form the words: the even lane
// stores the hi pairs, the odd lane the lo pairs.  Element pairs go through packed fp32 math
// (v_pk_fma / v_pk_add: per element the same fmaf and add).  Returns whether an accumulator
// was non-finite (their sum is: padding accumulators are exactly 0).  F32L (the last conv when
// the heads are fused): the block output goes to LDS as fp32 rows [pixel][128] instead of HBM.
// NJ (SPLIT: 1): the wave's 16-channel fragments, from fragment nb of its group.
template <bool RES, bool TO_LDS, int EABL = 0, bool F32L = false, int NJ = 2>
__device__ __forceinline__ bool b16_epilogue(const f32x4 (&acc)[5][NJ], const float* __restrict__ scale,
                                             const float* __restrict__ shift, __amdgpu_buffer_rsrc_t xr, char* lds,
                                             const int* poff, int mg, int cg, int lane, int nb = 0)
{
    asm volatile("" : "+v"(lane));   // the epilogue's addresses are rebuilt per conv, not hoisted (they would spill)
    const int r16 = lane & 15, kb = lane >> 4, odd = r16 & 1, ce = r16 & 14;
    // the lane's part of a store offset in a keyed row: slot (ce >> 3) ^ 4 (kb & 1), channel
    // ce & 7, lo half for the odd lane; the tile's 32 (n ^ (i >> 1)) and the row i * 128 are
    // immediates (row m = m0 + i has key 4 (kb & 1) | (i & 2))
    const int lpart = (16 * ((ce >> 3) ^ (4 * (kb & 1))) + 2 * (ce & 7)) ^ (odd ? 64 : 0);
    // the word of element i (e = 0) / i + 1 (e = 1) from X (own H or L) and Zp (the partner's):
    // even lane (own hi, partner hi), odd lane (partner lo, own lo)
    const unsigned sel0 = odd ? 0x01000504u : 0x05040100u, sel1 = odd ? 0x03020706u : 0x07060302u;
    float sc[NJ], sh[NJ];
#pragma unroll
    for (int nn = 0; nn < NJ; ++nn) {
        sc[nn] = scale[32 * cg + 16 * (nb + nn) + r16];
        sh[nn] = shift[32 * cg + 16 * (nb + nn) + r16];
    }
    const int cbyte = 4 * (32 * cg + r16);
    // every block-input load first (in program order ahead of the in-place stores, which the
    // compiler cannot move them past): one memory round trip per epilogue, not one per f
    int vof[5][4];
    float rvf[5][NJ][4];
    if constexpr (RES) {
#pragma unroll
        for (int f = 0; f < 5; ++f) {
            const int4 p4 = *(const int4*)(poff + 80 * mg + 16 * f + 4 * kb);
            vof[f][0] = p4.x + cbyte, vof[f][1] = p4.y + cbyte, vof[f][2] = p4.z + cbyte, vof[f][3] = p4.w + cbyte;
#pragma unroll
            for (int nn = 0; nn < NJ; ++nn)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    rvf[f][nn][i] = (EABL & 1) ? __builtin_bit_cast(float, vof[f][i])   // study: no residual loads
                                               : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                               xr, vof[f][i] + 64 * (nb + nn), 0, 0));
        }
    }
    b16_f32x2 chk = {0.f, 0.f};
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        const int m0 = 80 * mg + 16 * f + 4 * kb;
        const int (&vo)[4] = vof[f];
        const float (&rv)[NJ][4] = rvf[f];
        char* wrow = lds + kB16Act + (cg * kB16Rows + m0) * 128 + lpart;
#pragma unroll
        for (int nn = 0; nn < NJ; ++nn)
#pragma unroll
            for (int ip = 0; ip < 2; ++ip) {
                const int n = nb + nn;
                const b16_f32x2 v = {acc[f][nn][2 * ip], acc[f][nn][2 * ip + 1]};
                chk += v;
                b16_f32x2 y = __builtin_elementwise_fma(v, b16_f32x2{sc[nn], sc[nn]}, b16_f32x2{sh[nn], sh[nn]});
                if constexpr (RES) y += b16_f32x2{rv[nn][2 * ip], rv[nn][2 * ip + 1]};
                const float ye[2] = {fmaxf(y.x, 0.f), fmaxf(y.y, 0.f)};
                if constexpr (RES && F32L) {
#pragma unroll
                    for (int e = 0; e < 2; ++e)
                        if (f < 4 || m0 + 2 * ip + e < PIX)
                            *(float*)(lds + kB16Act + b16_f32_row(m0 + 2 * ip + e, 32 * cg + 16 * n + r16)) = ye[e];
                } else if constexpr (RES) {
#pragma unroll
                    for (int e = 0; e < 2; ++e)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, ye[e]), xr,
                                                              vo[2 * ip + e] + 64 * n, 0, 0);
                }
                if constexpr (TO_LDS) {
                    // the lane's two elements split together: H = (hi_i, hi_i+1), L = (lo_i, lo_i+1);
                    // the partner lane's H (to an even lane) or L (to an odd lane) by one DPP
                    // (lo = fp16(y - hi) by v_fma_mix{lo,hi}_f16: the exact fp32 difference rounded
                    // once to fp16, as the cvt / subtract / cvt sequence does)
                    const b16_f32x2 yy = {ye[0], ye[1]};
                    const b16_f16x2 hp = __builtin_convertvector(yy, b16_f16x2);
                    const unsigned H = __builtin_bit_cast(unsigned, hp);
                    unsigned L;
                    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
                        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                        : "=&v"(L) : "v"(H), "v"(ye[0]), "v"(ye[1]));
                    const unsigned X = odd ? L : H, Z = odd ? H : L;
                    const unsigned Zp = (unsigned)__builtin_amdgcn_mov_dpp((int)Z, 0xB1, 0xF, 0xF, false);
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int i = 2 * ip + e;
                        const unsigned word = __builtin_amdgcn_perm(Zp, X, e ? sel1 : sel0);
                        if (f < 4 || m0 + i < PIX)   // (padding rows past pixel 224 stay unwritten)
                            *(unsigned*)(wrow + i * 128 + 32 * (n ^ (i >> 1))) = word;
                    }
                }
            }
    }
    return !__builtin_isfinite(chk.x + chk.y);
}

// SPLIT: one wait of lane 0 on a neighbour's flag, bounded by the wave's AWAKE time (each
// s_memrealtime delta counts at most 10 us: a suspended dispatch does not time out on the
// gap), as pv_tower.hip's tower_wait.  Returns false on timeout.
__device__ __forceinline__ bool b16_wait(const unsigned* f, unsigned need, unsigned limit)
{
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need && limit != 0) return true;
    unsigned long long prev = __builtin_amdgcn_s_memrealtime();
    unsigned waited = 0;
    for (;;) {
        __builtin_amdgcn_s_sleep(2);
        const unsigned seen = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        const unsigned long long d = now - prev;
        prev = now;
        waited += d < 1000ull ? (unsigned)d : 1000u;
        if (seen >= need && limit != 0) return true;
        if (waited >= limit) return false;
    }
}

// SPLIT exchange after conv l (l + 1 < nlayers): workgroup mg owns pixels m0..m1-1 of the
// board; the next conv's taps read pixels up to 16 rows past them, so it publishes its first
// and last 16 pixel rows (every channel group: the LDS image's own keyed words, 16-B
// write-through stores, cdna_hip_programming.md Guideline 16 R1: drain, barrier, one agent-
// scope flag store), waits for the neighbours' flags, takes ONE agent-scope acquire, and
// copies their 16 rows next to its own.  Layer parity double-buffers the images: a neighbour
// cannot publish conv l + 2 before this workgroup published l + 1, i.e. finished reading l.
__device__ __forceinline__ void b16_exchange(const Board16Args& a, char* lds, int board, int mg, int l, int tid)
{
    char* xb = a.xbuf + ((size_t)board * 2 + (l & 1)) * kB16Img;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(xb, (short)0, kB16Img, 0x00020000);
    const int m0 = 80 * mg, m1 = mg == 2 ? PIX : m0 + 80;
    // piece p of the 1024 16-B pieces of two 16-row ranges (0: starting at lo, 1: at hi) x 4
    // groups -> byte offset in the image, -1 where the range has no neighbour
    auto piece = [&](int p, int lo, int hi) {
        const int r = p >> 9, q = p & 511, g = q >> 7, row = (q >> 3) & 15;
        if (r == 0 ? mg == 0 : mg == 2) return -1;
        return (g * kB16Rows + (r == 0 ? lo : hi) + row) * 128 + 16 * (q & 7);
    };
#pragma unroll
    for (int k = 0; k < 1024 / kB16SplitThreads; ++k) {
        const int o = piece(tid + kB16SplitThreads * k, m0, m1 - 16);
        if (o >= 0) __builtin_amdgcn_raw_buffer_store_b128(*(const b16_u32x4*)(lds + kB16Act + o), xr, o, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        unsigned* fl = a.xflag + (size_t)board * 3;
        const unsigned tag = a.epoch * 64u + (unsigned)l + 1u;
        __hip_atomic_store(fl + mg, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
        if (mg > 0) ok = b16_wait(fl + mg - 1, tag, a.limit) && ok;
        if (mg < 2) ok = b16_wait(fl + mg + 1, tag, a.limit) && ok;
        if (!ok) {   // the rows are stale: post the launch (azg_pv_recover reruns it unsplit) and go on
            if (a.ring && a.seq)
                __hip_atomic_store(a.ring + (a.seq & (kTowerRing - 1)), a.seq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            if (a.diag) __hip_atomic_fetch_add(a.diag + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    constexpr int K = 1024 / kB16SplitThreads;
    b16_u32x4 v[K];
    int off[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        off[k] = piece(tid + kB16SplitThreads * k, m0 - 16, m1);
        if (off[k] >= 0) v[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, off[k], 0, 0);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (off[k] >= 0) *(b16_u32x4*)(lds + kB16Act + off[k]) = v[k];
    __syncthreads();
}

extern int g_board_abl;
// ABL: timing ablations of the study build (key 51): 1 no DMA wait, 2 no barrier, 4 no epilogue
// (the accumulators kept live), 8 fixed A rows, 64 no residual loads; the product runs ABL 0
// SPLIT (small batches): three 8-wave workgroups per board, workgroup 3 b + mg computing pixels
// 80 mg .. 80 mg + 79 of every channel (wave = one 16-channel fragment: 80x16 tiles), the same
// per-element MFMA chains (bitwise the unsplit tower), conv outputs' boundary rows exchanged
// through L2 (b16_exchange); the tower output goes to x (the heads run unfused).
template <int ABL, bool SPLIT = false>
__global__ __launch_bounds__(SPLIT ? kB16SplitThreads : kB16Threads, 1) void board16_tower(const Board16Args a)
{
    constexpr int NT = SPLIT ? kB16SplitThreads : kB16Threads;
    constexpr int NJ = SPLIT ? 1 : 2;   // 16-channel fragments per wave
    extern __shared__ __attribute__((aligned(16))) float smem_f[];
    char* lds = (char*)smem_f;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // SPLIT: wave w computes channel group w / 2, its 16-channel fragment w % 2
    const int mg = SPLIT ? (int)blockIdx.x % 3 : wid % 3, ng = SPLIT ? wid >> 1 : wid / 3, nb = SPLIT ? wid & 1 : 0;
    const int r16 = lane & 15, kb = lane >> 4;
    int* poff = (int*)(lds + kB16Prow);   // byte offset of each pixel's padded row (padding: past the board)

    // padded row of every pixel (-1 past pixel 224), the groups' zero rows
    for (int i = tid; i < 240; i += NT)
        poff[i] = i < PIX ? ((i / BOARD + 1) * PADW + i % BOARD + 1) * kB16C * 4 : 0x40000000;
    if (tid < kB16Groups * 32) ((float*)(lds + kB16Act + ((tid >> 5) * kB16Rows + PIX) * 128))[tid & 31] = 0.f;
    if (a.hout)
        for (int i = tid; i < 3 * kB16C; i += NT) ((float*)(lds + kB16Hw))[i] = i < 2 * kB16C ? a.hwp[i] : a.hwv[i - 2 * kB16C];

    // this lane's A rows (pixel 80 mg + 16 f + r16 of fragment f) and the taps on the board
    int pf[5];
    unsigned tm[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        const int p = 80 * mg + 16 * f + r16;
        const int py = p / BOARD, px = p - py * BOARD;
        unsigned t = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int yy = py + k / 3 - 1, xx = px + k % 3 - 1;
            if (p < PIX && yy >= 0 && yy < BOARD && xx >= 0 && xx < BOARD) t |= 1u << k;
        }
        pf[f] = p;
        tm[f] = t;
    }
    // B fragments: weight row n = 32 ng + 16 j + r16, slot kb (hi) / kb ^ 4 (lo), keyed by n & 6 = r16 & 6
    const int bh0 = (32 * ng + 16 * nb + r16) * 128 + 16 * (kb ^ (r16 & 6));
    const int bl0 = bh0 ^ 64;

    // weight DMA of one chunk (16 KB, 128 rows x 128 B): wave w moves rows 8 w .. 8 w + 7,
    // waves 0..3 also rows 96 + 8 w ..; lane -> row + lane / 8, LDS slot lane % 8 holding
    // source slot (lane % 8) ^ (row & 6)
    const int wr0 = 8 * wid + (lane >> 3);
    const int ws0 = wr0 * 32 + (((lane & 7) ^ (wr0 & 6)) * 4);
    const int wr1 = 96 + 8 * (wid & 3) + (lane >> 3);
    const int ws1 = wr1 * 32 + (((lane & 7) ^ (wr1 & 6)) * 4);
    auto dma = [&](const float* wl, int s, int buf) {   // chunk s = cg * 9 + tap -> stage buf
        const int cg = s / 9, tap = s - cg * 9;
        const float* src = wl + (size_t)(tap * kB16Groups + cg) * kB16C * 32;
        if constexpr (SPLIT) {   // 8 waves: rows 8 (w + 8 k) .. + 7 (row & 6 as for k = 0)
#pragma unroll
            for (int k = 0; k < 2; ++k)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + ws0 + 2048 * k),
                                                 (__attribute__((address_space(3))) void*)(lds + buf * kB16Stage +
                                                                                           (wid + 8 * k) * 1024),
                                                 16, 0, 0);
        } else {
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + ws0),
                                             (__attribute__((address_space(3))) void*)(lds + buf * kB16Stage + wid * 1024),
                                             16, 0, 0);
            if (wid < 4)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + ws1),
                                                 (__attribute__((address_space(3))) void*)(lds + buf * kB16Stage + (12 + wid) * 1024),
                                                 16, 0, 0);
        }
    };

    const int nl = a.nlayers;
    int board = SPLIT ? (int)blockIdx.x / 3 : (int)blockIdx.x;
    const int bstride = SPLIT ? a.B : (int)gridDim.x;
    if (board < a.B) {   // the first conv's chunks 0 and 1
        dma(a.wp[0], 0, 0);
        dma(a.wp[0], 1, 1);
    }
    __syncthreads();   // poff / zero rows
    for (; board < a.B; board += bstride) {
        float* xb = a.x + (size_t)board * PADPIX * kB16C;
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(xb, (short)0, PADPIX * kB16C * 4, 0x00020000);
        int t8 = tid;
        asm volatile("" : "+v"(t8));   // the staging addresses are rebuilt per board, not kept live
        // ---- the board's stem output -> hi / lo rows [group][pixel], in two halves of 5
        // float4 per thread (all 10 in flight at once would spill) ----
#pragma unroll
        for (int half = 0; half < (PIX * 32 + 5 * NT - 1) / (5 * NT); ++half) {
            constexpr int kIt = 5;
            f32x4 v[kIt];
#pragma unroll
            for (int k = 0; k < kIt; ++k) {
                const int i = t8 + (half * kIt + k) * NT;   // (pixel, float4 of 128 channels)
                if (i < PIX * 32) v[k] = *(const f32x4*)((const char*)xb + poff[i >> 5] + (i & 31) * 16);
            }
#pragma unroll
            for (int k = 0; k < kIt; ++k) {
                const int i = t8 + (half * kIt + k) * NT;
                if (i < PIX * 32) {
                    const int m = i >> 5, c4 = i & 31, g = c4 >> 3, q4 = c4 & 7;
                    f16x4 hi, lo;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        hi[e] = (_Float16)v[k][e];
                        lo[e] = (_Float16)(v[k][e] - (float)hi[e]);
                    }
                    char* row = lds + kB16Act + (g * kB16Rows + m) * 128;
                    const int o = 16 * ((q4 >> 1) ^ (m & 6)) + (q4 & 1) * 8;
                    *(f16x4*)(row + o) = hi;
                    *(f16x4*)(row + (o ^ 64)) = lo;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of the first chunks
        __syncthreads();
        const bool more_boards = board + bstride < a.B;

        for (int l = 0; l < nl; ++l) {
            f32x4 acc[5][NJ];
#pragma unroll
            for (int f = 0; f < 5; ++f)
#pragma unroll
                for (int n = 0; n < NJ; ++n) acc[f][n] = f32x4{0.f, 0.f, 0.f, 0.f};
            // this conv's and the next one's weights (scalar, loaded once per conv); the next
            // conv's chunks 0 and 1 are issued during steps 34 and 35
            const float* wl = a.wp[l];
            const float* wn = l + 1 < nl ? a.wp[l + 1] : a.wp[0];
            const bool more = l + 1 < nl || more_boards;
            // A rows of (cg, tap) for fragment f: neighbour pixel q (the group's zero row off
            // the board), rebuilt per tap (45 hoisted row addresses would not fit)
            auto arow = [&](int cg, int tap, int f) {
                if constexpr ((ABL & 8) != 0) return kB16Act + (cg * kB16Rows + pf[f]) * 128 + 16 * (kb ^ (pf[f] & 6));
                asm volatile("" : "+v"(tm[f]), "+v"(pf[f]));
                const int d = (tap / 3 - 1) * BOARD + (tap % 3 - 1);
                const int q = ((tm[f] >> tap) & 1) ? pf[f] + d : PIX;
                return kB16Act + (cg * kB16Rows + q) * 128 + 16 * (kb ^ (q & 6));
            };
            // step 0's operands; then every wave holds chunk 0's B fragments and stage 0 may
            // be refilled
            f16x8 bh[NJ], bl[NJ], ah[5], al[5];
#pragma unroll
            for (int f = 0; f < 5; ++f) {
                const int ao = arow(0, 0, f);
                al[f] = *(const f16x8*)(lds + (ao ^ 64));
                ah[f] = *(const f16x8*)(lds + ao);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                bh[j] = *(const f16x8*)(lds + bh0 + j * 2048);
                bl[j] = *(const f16x8*)(lds + bl0 + j * 2048);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __syncthreads();
            // K32 step s = 9 cg + tap computes from registers read during step s - 1: chunk
            // s + 1 was published by the barrier ending step s - 1 and the conv's input is
            // static, so step s + 1's fragments are read between this step's product groups
            // (each into the registers its group just released); chunk s + 2 is issued into
            // the stage chunk s used (read during step s - 1: every wave is past it)
            for (int cg = 0; cg < kB16Groups; ++cg) {
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    const int s = cg * 9 + tap;
                    const int buf = (cg + tap) & 1;   // = s & 1
                    if (tap < 7 || cg + 1 < kB16Groups) dma(wl, s + 2, buf);
                    else if (more) dma(wn, s + 2 - kB16Steps, buf);
                    const bool nx = tap < 8 || cg + 1 < kB16Groups;   // (scalar)
                    const int ncg = tap < 8 ? cg : cg + 1, ntap = tap < 8 ? tap + 1 : 0;
                    const char* bn = lds + (buf ^ 1) * kB16Stage;
                    // per element the chain lo_a hi_b, hi_a hi_b, hi_a lo_b, product-major over
                    // the 10 tiles (no MFMA waits on the one before)
#pragma unroll
                    for (int f = 0; f < 5; ++f)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[f], bh[j], acc[f][j], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    int ao[5];
                    if (nx) {
#pragma unroll
                        for (int f = 0; f < 5; ++f) {
                            ao[f] = arow(ncg, ntap, f);
                            al[f] = *(const f16x8*)(lds + (ao[f] ^ 64));
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int f = 0; f < 5; ++f)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[f], bh[j], acc[f][j], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    if (nx) {
#pragma unroll
                        for (int j = 0; j < NJ; ++j) bh[j] = *(const f16x8*)(bn + bh0 + j * 2048);
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int f = 0; f < 5; ++f)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[f], bl[j], acc[f][j], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    if (nx) {   // the B reads first: the barrier need only wait for them
#pragma unroll
                        for (int j = 0; j < NJ; ++j) bl[j] = *(const f16x8*)(bn + bl0 + j * 2048);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int f = 0; f < 5; ++f) ah[f] = *(const f16x8*)(lds + ao[f]);
                    }
                    // chunk s + 2 has landed (this wave's pieces); the barrier publishes it for
                    // step s + 1's reads, and every wave's reads of chunk s + 1 are complete (its
                    // stage takes chunk s + 3)
                    // (the barrier waits for this wave's B reads of chunk s + 1, issued before its
                    // A reads: the 5 activation reads may stay in flight -- no DMA writes there)
                    if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(5)" ::: "memory");
                    if constexpr (!(ABL & 2)) __builtin_amdgcn_s_barrier();
                }
            }

            // ---- epilogue: BN (+ block input) + ReLU; every wave is past its last read of
            // this conv's input (the barrier above) ----
            const float *sc = a.scale[l], *sh = a.shift[l];
            bool bad = false;
            if (ABL & 4) {
                float t = 0.f;
#pragma unroll
                for (int f = 0; f < 5; ++f)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) t += acc[f][j][0] + acc[f][j][1] + acc[f][j][2] + acc[f][j][3];
                if (t == 1234.5f) xb[tid] = t;
            }
            else if (!(l & 1))
                bad = b16_epilogue<false, true, (ABL >> 6), false, NJ>(acc, sc, sh, xr, lds, poff, mg, ng, lane, nb);
            else if (l + 1 < nl)
                bad = b16_epilogue<true, true, (ABL >> 6), false, NJ>(acc, sc, sh, xr, lds, poff, mg, ng, lane, nb);
            else if (!SPLIT && a.hout)
                bad = b16_epilogue<true, false, (ABL >> 6), true, NJ>(acc, sc, sh, xr, lds, poff, mg, ng, lane, nb);
            else bad = b16_epilogue<true, false, (ABL >> 6), false, NJ>(acc, sc, sh, xr, lds, poff, mg, ng, lane, nb);
            if (bad && a.ring_ovf && a.seq)
                __hip_atomic_store(a.ring_ovf + (a.seq & (kTowerRing - 1)), a.seq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            // the next conv reads what every wave wrote to LDS.  The block-output stores need
            // not land first: only this lane reads them back (the residual two convs on, and
            // a wave's memory operations to one address stay in order), and the next step's
            // vmcnt(0) retires them behind step 0's MFMAs
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if constexpr (SPLIT)
                if (l + 1 < nl) b16_exchange(a, lds, board, mg, l, tid);
        }
        if (!SPLIT && a.hout) {
            // the heads' three 1x1 projections of the tower output (network.py:102-103, 110-111)
            // from the fp32 rows in LDS, heads_project's arithmetic (pv_heads.hip): lane 4 m + q
            // chains channels 32 q .. 32 q + 31, two xor shuffles sum the quarters, then BN + ReLU
            float* hb = a.hout + (size_t)board * FC_FS;
            int tp = tid;
            asm volatile("" : "+v"(tp));   // addresses rebuilt per board, not kept live across the convs
            for (int i0 = 0; i0 < PIX * 4; i0 += kB16Threads) {
                const int i = i0 + tp, m = i >> 2, q = i & 3;
                float d0 = 0.f, d1 = 0.f, d2 = 0.f;
                if (m < PIX) {
                    const float* w0 = (const float*)(lds + kB16Hw) + 32 * q;
                    const float *w1 = w0 + kB16C, *w2 = w0 + 2 * kB16C;
#pragma unroll
                    for (int c = 0; c < 32; c += 4) {
                        const f32x4 v = *(const f32x4*)(lds + kB16Act + b16_f32_row(m, 32 * q + c));
                        const f32x4 u0 = *(const f32x4*)(w0 + c), u1 = *(const f32x4*)(w1 + c),
                                    u2 = *(const f32x4*)(w2 + c);
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            d0 = fmaf(v[k], u0[k], d0);
                            d1 = fmaf(v[k], u1[k], d1);
                            d2 = fmaf(v[k], u2[k], d2);
                        }
                    }
                }
#pragma unroll
                for (int o = 1; o < 4; o <<= 1) {
                    d0 += __shfl_xor(d0, o, 64);
                    d1 += __shfl_xor(d1, o, 64);
                    d2 += __shfl_xor(d2, o, 64);
                }
                if (m < PIX && q == 0) {
                    hb[m] = head_bn_relu(d0, a.hsc[0], a.hsh[0]);
                    hb[PIX + m] = head_bn_relu(d1, a.hsc[1], a.hsh[1]);
                    hb[FC_KP + m] = head_bn_relu(d2, a.hsc[2], a.hsh[2]);
                }
            }
            __syncthreads();   // the rows are read before the next board's stem output lands there
            // the fp32 rows covered the groups' zero rows: restore them
            if (tp < kB16Groups * 32) ((float*)(lds + kB16Act + ((tp >> 5) * kB16Rows + PIX) * 128))[tp & 31] = 0.f;
        }
    }
}

int g_board16_split = 85;   // key 52: largest batch run split (three workgroups per board, 3 B <= CUs); 0: never
static int g_b16_cus = 0, g_b16_grid = 0;

// first use: the kernels' dynamic LDS attribute, the one-per-CU grid and the CU count
static hipError_t b16_init()
{
    if (g_b16_grid) return hipSuccess;
    hipError_t e = hipSuccess;
#ifdef AZG_AB_STUDIES
    for (const void* f : {(const void*)board16_tower<0>, (const void*)board16_tower<3>, (const void*)board16_tower<4>,
                          (const void*)board16_tower<8>, (const void*)board16_tower<15>,
                          (const void*)board16_tower<64>, (const void*)board16_tower<0, true>})
#else
    for (const void* f : {(const void*)board16_tower<0>, (const void*)board16_tower<0, true>})
#endif
        if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kB16Lds)) != hipSuccess) return e;
    int per_cu = 0, dev = 0, cus = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)board16_tower<0>, kB16Threads, kB16Lds);
    if (e != hipSuccess) return e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if (per_cu < 1) return hipErrorInvalidConfiguration;
    g_b16_cus = cus;
    g_b16_grid = per_cu * cus;
    return hipSuccess;
}

int board16_grid()
{
    return b16_init() == hipSuccess ? g_b16_grid : 0;
}

int board16_split_max()
{
    if (b16_init() != hipSuccess) return 0;
    const int m = g_b16_cus / 3 < kB16SplitCap ? g_b16_cus / 3 : kB16SplitCap;
    return g_board16_split < m ? g_board16_split : m;
}

hipError_t launch_board16_tower(int NB, const float* wp16, const float* scale16, const float* shift,
                                const int* out_off, float* x, int B, unsigned* ring_ovf, unsigned seq, hipStream_t st,
                                const float* hwp, const float* hwv, const float* hsc, const float* hsh, float* hout,
                                const Board16Split* sp)
{
    if (2 * NB > kB16MaxLayers || NB <= 0 || B <= 0) return hipErrorInvalidValue;
    if (hipError_t e = b16_init()) return e;
    const int grid = g_b16_grid;
    Board16Args a{};
    for (int l = 0; l < 2 * NB; ++l) {
        a.wp[l] = wp16 + (size_t)l * 9 * kB16C * kB16C;
        a.scale[l] = scale16 + out_off[l];
        a.shift[l] = shift + out_off[l];
    }
    a.x = x;
    a.B = B;
    a.nlayers = 2 * NB;
    a.ring_ovf = ring_ovf;
    a.seq = seq;
    if (hout && !(hwp && hwv && hsc && hsh)) return hipErrorInvalidValue;
    a.hwp = hwp, a.hwv = hwv, a.hsc = hsc, a.hsh = hsh, a.hout = hout;
    if (sp) {   // three workgroups per board, all resident (one per CU): B <= CUs / 3
        if (hout || 3 * B > g_b16_cus) return hipErrorInvalidValue;
        a.xbuf = sp->xbuf, a.xflag = sp->xflag, a.epoch = sp->epoch, a.ring = sp->ring, a.diag = sp->diag;
        a.limit = g_tower_wait_us >= 0xffffffffu / 100u ? 0xffffffffu : g_tower_wait_us * 100u;
        hipLaunchKernelGGL((board16_tower<0, true>), dim3(3 * B), dim3(kB16SplitThreads), kB16Lds, st, a);
        return hipGetLastError();
    }
    const dim3 g(B < grid ? B : grid);
#ifdef AZG_AB_STUDIES
    switch (g_board_abl) {   // timing ablations (key 51, study build; results invalid while set)
        case 3: hipLaunchKernelGGL(board16_tower<3>, g, dim3(kB16Threads), kB16Lds, st, a); return hipGetLastError();
        case 4: hipLaunchKernelGGL(board16_tower<4>, g, dim3(kB16Threads), kB16Lds, st, a); return hipGetLastError();
        case 8: hipLaunchKernelGGL(board16_tower<8>, g, dim3(kB16Threads), kB16Lds, st, a); return hipGetLastError();
        case 15: hipLaunchKernelGGL(board16_tower<15>, g, dim3(kB16Threads), kB16Lds, st, a); return hipGetLastError();
        case 64: hipLaunchKernelGGL(board16_tower<64>, g, dim3(kB16Threads), kB16Lds, st, a); return hipGetLastError();
        default: break;
    }
#endif
    hipLaunchKernelGGL(board16_tower<0>, g, dim3(kB16Threads), kB16Lds, st, a);
    return hipGetLastError();
}

}  // namespace azg
