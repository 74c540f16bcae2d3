// Persistent residual-tower kernel: every 3x3 conv of the eval forward's tower
// (network.py:98-99, ResidualBlock network.py:9-26) in ONE launch.
//
// Why: a per-layer launch ends with a partial round of tiles (at B = 512, 3600
// 64x64 tiles on 1024 resident slots) and every layer waits for the previous one
// to drain.  Here workgroups stay resident and claim tiles (layer-major, then M
// tile, then N tile) from one atomic counter; tile (l, mt) starts as soon as the
// three layer-(l-1) M tiles whose rows its halo reads (mt-1, mt, mt+1) are done, so
// the tail of one layer overlaps the head of the next.
//
// Tile body: halo_tile (pv_halo.h), identical arithmetic to the per-layer kernel
// (results are bitwise equal to the per-layer path).
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md
// "Valid forms"), producer side always R1: every output element is stored
// write-through (16-B buffer_store sc1); each wave drains (s_waitcnt vmcnt(0));
// workgroup barrier; one lane adds the tile count to the (layer, M tile) counter
// with an agent-scope atomic.  Consumer: one lane polls the (up to) three counters
// with relaxed agent-scope loads (global_load sc1) until each is complete, then
//  * VAR bit 16 clear (64x64 / 128x64 tiles, 2-4 workgroups per CU): ONE agent-scope
//    acquire, s_waitcnt vmcnt(0), workgroup barrier, plain loads -- the form valid at
//    any occupancy;
//  * VAR bit 16 set (the 16-wave 128x128 tile, exactly ONE workgroup per CU, checked
//    at launch): s_waitcnt vmcnt(0), workgroup barrier, and EVERY load of handed-off
//    bytes (halo rows, the epilogue's residual) is a 16-B sc1 buffer load -- row 1 of
//    the guide's measured hand-off table, which requires one workgroup per CU in
//    every cell; no LDS-DMA or early-epilogue path may be combined with it
//    (static_assert below).
// Deadlock freedom: a tile waits only on tiles claimed before it (all of layer
// l-1 precedes layer l in claim order), and a claimed tile is always executed by a
// running workgroup, so the oldest unfinished tile can always finish.  Waits are
// bounded by the waiting wave's AWAKE time (tower_wait below); a timeout posts the
// launch's sequence number to the handle's host ring (azg_pv_recover recomputes that
// forward per layer), fills the self-describing record (azg_pv_tower_diag) and the
// workgroup proceeds so the grid always drains.
//
// Buffer reuse (WAR): with X -> H -> Y(+X) -> H -> X(+Y) ..., a tile overwrites
// rows whose readers are exactly (or transitively) the tiles it waits on.
#include "pv_internal.h"
#include "pv_halo.h"
#include "pv_h3.h"

namespace azg {

constexpr int kTowerMaxLayers = 2 * kTowerMaxBlocks;

struct TowerLayer {
    const float* wp;
    const float* scale;
    const float* shift;
    const float* in;
    const float* resid;    // nullptr for the first conv of a block
    float* out;
};

struct TowerArgs {
    TowerLayer L[kTowerMaxLayers];
    int nlayers;
    int M;
    int act_bytes;       // bytes of one activation buffer (buffer descriptor range)
    unsigned* sync;      // [0] work counter, [1] error word, [4..] per-(layer, M tile) counters
    unsigned* ring;      // host-mapped ring of timed-out launch numbers (azg_pv_recover); may be null
    unsigned* ring_ovf;  // host-mapped ring of H3 launches whose activations left fp16's range
    unsigned* diag;      // persistent wait record (TowerDiag layout, azg_pv_tower_diag); may be null
    uint4* prod;         // per (layer, M tile): {seq, HW_ID, XCC_ID, start tick} of the workgroup running it
    unsigned seq;        // launch sequence number (0: autotuning runs, never posted)
    unsigned limit;      // awake-time bound of one dependency wait, in 10-ns ticks (0: time out at once)
    int group;           // 1: a claim is one (M, N) tile; NTN: one M tile with all its N
                         // tiles, run back to back by the claiming workgroup (the second
                         // N tile's halo rows are hits in that XCD's L2)
    int abl;             // timing studies only (0 in the product; results not valid otherwise):
                         // bit 1 skips the dependency wait + acquire, bit 2 the publish drain
};

unsigned g_tower_wait_us = kTowerWaitUs;     // tuning key 14 (tests: 0 forces the timeout path)
int g_tower_group = 1;                       // tuning key 17: 1 (default) = claim an M tile with all its N tiles
#ifdef AZG_AB_STUDIES
int g_tower_coh = 0;   // study key 31: sc1 dependent loads with 64x64 / 128x64 tiles (OUTSIDE the guide's envelope)
#endif

// waves per SIMD the register budget is sized for: 4 (128 VGPRs) for the one-
// accumulator tiles (two 8-wave or four 4-wave workgroups per CU, or the one 16-wave
// workgroup); 2 (256 VGPRs, one 8-wave workgroup per CU) for 128-wide N tiles of 8 waves
template <int BN_, int NW_>
constexpr int tower_min_waves() { return NW_ >= 16 ? 4 : BN_ >= 128 ? 2 : 4; }
// dynamic LDS of a tower launch: the 16-wave tile asks for more than half of the CU's
// 160 KiB so that one workgroup per CU is guaranteed by LDS alone (the sc1-load
// hand-off is valid only there), whatever the register allocation
// VAR bit 256: the tile body is h3_tile (pv_h3.h: split-fp16, LDS-DMA weight stages of one
// tap, three stage buffers), else halo_tile
constexpr int kH3TileTps = 1, kH3TileNwb = 3;
template <int C, int BN, int WM, int TM, int NW, int VAR>
constexpr int tower_body_lds()
{
    if constexpr ((VAR & 256) != 0) return H3Tile<C, BN, WM, TM, NW, kH3TileTps, kH3TileNwb>::LDS;
    else return halo_lds_bytes<C, BN, WM, TM, NW, VAR & 255>();
}
template <int C, int BN, int WM, int TM, int NW, int VAR>
constexpr int tower_lds_bytes()
{
    constexpr int need = tower_body_lds<C, BN, WM, TM, NW, VAR>() + 16;
    return NW >= 16 && need <= 82 * 1024 ? 82 * 1024 : need;
}

// Device side of azg_pv_tower_diag (word offsets into a.diag; the host converts ticks
// to microseconds).
enum TowerDiag : int {
    TD_TAKEN = 0,         // 0 until the first timed-out wait claims the record
    TD_TIMEOUTS, TD_W100US, TD_W1MS, TD_W10MS, TD_W100MS, TD_MAXWAIT,
    TD_SEQ, TD_LAYER, TD_MTILE, TD_WAIT_MTILE, TD_OBSERVED, TD_NEEDED, TD_WAITED, TD_WALL,
    TD_WAITER_HW, TD_WAITER_XCC, TD_CLAIMS, TD_PCLAIMED, TD_PSTARTED, TD_PHW, TD_PXCC, TD_PSTART,
    TD_MAXWALL,           // longest wall time of a wait (awake + suspended)
    TD_SUSP,              // waits whose wall time exceeded their awake time by > 1 ms (the wave was suspended)
    TD_WORDS
};
static_assert(TD_WORDS <= kTowerDiagWords, "tower diag record");

__device__ __forceinline__ unsigned hw_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}
__device__ __forceinline__ unsigned xcc_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 15u;
}

// One dependency wait (lane 0 of the waiting workgroup): relaxed agent-scope polls
// with s_sleep between them until the counter reaches `need`.  The bound is the
// wave's AWAKE time: each s_memrealtime delta (100 MHz) counts at most kWaitStep
// ticks, so a wave that was context-saved together with its producer (queue
// preemption suspends every wave of the dispatch) does not time out on the gap.
// The fast path (counter already complete) reads no clock.  Returns false on timeout.
constexpr unsigned kWaitStep = 1000;   // 10 us
__device__ __forceinline__ bool tower_wait(const unsigned* c, unsigned need, unsigned limit, unsigned& seen,
                                           unsigned& waited, unsigned long long& t0, unsigned long long& t1)
{
    seen = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    waited = 0;
    if (seen >= need && limit != 0) return true;
    t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long prev = t0;
    for (;;) {
        __builtin_amdgcn_s_sleep(2);
        seen = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        const unsigned long long d = now - prev;
        prev = now;
        waited += d < kWaitStep ? (unsigned)d : kWaitStep;
        t1 = now;
        if (seen >= need && limit != 0) return true;
        if (waited >= limit) return false;
    }
}

// Book-keeping of a wait that took `waited` awake ticks over `wall` ticks of wall time
// (only slow waits get here)
__device__ __forceinline__ void tower_wait_stats(unsigned* d, unsigned waited, unsigned wall)
{
    if (!d) return;
    __hip_atomic_fetch_max(d + TD_MAXWALL, wall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wall - waited > 100000u) __hip_atomic_fetch_add(d + TD_SUSP, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (waited > 10000u) __hip_atomic_fetch_add(d + TD_W100US, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (waited > 100000u) __hip_atomic_fetch_add(d + TD_W1MS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (waited > 1000000u) __hip_atomic_fetch_add(d + TD_W10MS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (waited > 10000000u) __hip_atomic_fetch_add(d + TD_W100MS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (waited > 10000u) __hip_atomic_fetch_max(d + TD_MAXWAIT, waited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A timed-out wait of tile (l, mt) on tile (l - 1, j): post the launch to the host
// ring and, if first since the record was cleared, describe it -- including what the
// producer tile's workgroup had published about itself in this launch.
__device__ __noinline__ void tower_timeout(unsigned* ring, unsigned* d, const unsigned* sync, const uint4* prod,
                                              unsigned seq, int l, int mt, int j, int mtiles, int tpl, unsigned seen,
                                              unsigned need, unsigned waited, unsigned long long t0,
                                              unsigned long long t1)
{
    if (ring && seq)
        __hip_atomic_store(ring + (seq & (kTowerRing - 1)), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!d) return;
    __hip_atomic_fetch_add(d + TD_TIMEOUTS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned zero = 0;
    if (!__hip_atomic_compare_exchange_strong(d + TD_TAKEN, &zero, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT))
        return;
    auto ld = [](const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto st = [&](int k, unsigned v) { __hip_atomic_store(d + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    const unsigned claims = ld(sync);
    const unsigned* pp = (const unsigned*)(prod + (size_t)(l - 1) * mtiles + j);
    const bool started = ld(pp) == seq;
    // claim index of the producer's (first) claim: layer-major, then M tile
    const unsigned pidx = (unsigned)((l - 1) * tpl + j * (tpl / mtiles));
    st(TD_SEQ, seq);
    st(TD_LAYER, (unsigned)l);
    st(TD_MTILE, (unsigned)mt);
    st(TD_WAIT_MTILE, (unsigned)j);
    st(TD_OBSERVED, seen);
    st(TD_NEEDED, need);
    st(TD_WAITED, waited);
    st(TD_WALL, (unsigned)(t1 - t0));
    st(TD_WAITER_HW, hw_id());
    st(TD_WAITER_XCC, xcc_id());
    st(TD_CLAIMS, claims);
    st(TD_PCLAIMED, claims > pidx ? 1u : 0u);
    st(TD_PSTARTED, started ? 1u : 0u);
    st(TD_PHW, started ? ld(pp + 1) : 0u);
    st(TD_PXCC, started ? ld(pp + 2) : 0u);
    st(TD_PSTART, started ? ld(pp + 3) - (unsigned)t0 : 0u);   // signed on the host
}

// HABL (study build, timing / traffic ablations only: results invalid): halo_tile's ABL
// bits -- 1 skips the weight loads, 2 the halo loads
template <int C, int BN_, int WM_, int TM_, int NW_, int VAR = 0, int HABL = 0>
__global__ __launch_bounds__(64 * NW_, (tower_min_waves<BN_, NW_>())) void conv_tower(const TowerArgs a)
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    static_assert(!((VAR & 48) && (VAR & 12)), "buffer halo / residual loads (VAR 16, 32) exclude LDS-DMA (4) and early epilogue loads (8)");
    constexpr int NTN = C / T::BN;
    constexpr int LDS_FLOATS = tower_body_lds<C, BN_, WM_, TM_, NW_, VAR>() / 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int* s_claim = (int*)(smem + LDS_FLOATS);

    const int tid = threadIdx.x;
    const int mtiles = (a.M + T::BM - 1) / T::BM;
    const int grp = a.group;                     // N tiles per claim (1 or NTN)
    const int tpl = mtiles * (NTN / grp);        // claims per layer
    const int total = tpl * a.nlayers;
    unsigned* work = a.sync;
    unsigned* err = a.sync + 1;
    unsigned* cnt = a.sync + 4;

    if (tid == 0) s_claim[0] = (int)__hip_atomic_fetch_add(work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    // the claim is workgroup-uniform: keep it (and the layer / tile indices and the
    // layer's pointers derived from it) in scalar registers
    int w = __builtin_amdgcn_readfirstlane(s_claim[0]);
    while (w < total) {
        const int l = w / tpl, t = w - l * tpl;
        const int mt = t / (NTN / grp), nt0 = (t - mt * (NTN / grp)) * grp;
        __syncthreads();                          // every wave has read s_claim
        if (tid == 0) {
            // next claim now: its latency overlaps this tile (read after the tile)
            s_claim[0] = (int)__hip_atomic_fetch_add(work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (l > 0 && !(a.abl & 1)) {
                const unsigned* c = cnt + (size_t)(l - 1) * mtiles;
                const int j0 = max(mt - 1, 0), j1 = min(mt + 1, mtiles - 1);
                for (int j = j0; j <= j1; ++j) {
                    unsigned seen, waited;
                    unsigned long long t0 = 0, t1 = 0;
                    if (!tower_wait(c + j, (unsigned)NTN, a.limit, seen, waited, t0, t1)) {
                        // the tile computes on stale inputs: flag the launch (the host
                        // recomputes it per layer) and describe the wait
                        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        tower_timeout(a.ring, a.diag, a.sync, a.prod, a.seq, l, mt, j, mtiles, tpl, seen, (unsigned)NTN,
                                      waited, t0, t1);
                    }
                    if (waited > 10000u || t1 - t0 > 10000u) tower_wait_stats(a.diag, waited, (unsigned)(t1 - t0));
                }
                // VAR bit 16 (one workgroup per CU): every dependent read is an sc1 load,
                // no acquire; otherwise ONE agent-scope acquire (L1 invalidate) here
                if constexpr ((VAR & 16) == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // what this tile's workgroup publishes about itself (read only by a timed-out
            // waiter's record): one 16-B store per claim
            if (a.prod) {
                const uint4 pr = make_uint4(a.seq, hw_id(), xcc_id(), (unsigned)__builtin_amdgcn_s_memrealtime());
                __hip_atomic_store((unsigned*)(a.prod + (size_t)l * mtiles + mt) + 1, pr.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned*)(a.prod + (size_t)l * mtiles + mt) + 2, pr.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned*)(a.prod + (size_t)l * mtiles + mt) + 3, pr.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned*)(a.prod + (size_t)l * mtiles + mt) + 0, pr.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        const TowerLayer& Ly = a.L[l];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Ly.out, (short)0, a.act_bytes, 0x00020000);
        for (int nt = nt0; nt < nt0 + grp; ++nt) {
            if (nt > nt0) __syncthreads();        // the previous tile's epilogue is done with LDS
            if constexpr ((VAR & 256) != 0)
                h3_tile<C, BN_, WM_, TM_, NW_, kH3TileTps, kH3TileNwb, EPI_BN_OPTRES_RELU, true, 1>(
                    Ly.in, Ly.wp, Ly.scale, Ly.shift, Ly.resid, Ly.out, rs, a.M, mt * T::BM, nt * T::BN, smem,
                    H3Guard{a.ring_ovf, a.seq});
            else
                halo_tile<C, BN_, WM_, TM_, NW_, EPI_BN_OPTRES_RELU, true, HABL, VAR>(
                    Ly.in, Ly.wp, Ly.scale, Ly.shift, Ly.resid, Ly.out, rs, a.M, mt * T::BM, nt * T::BN, smem, EpiX{},
                    ProX{}, FinX{}, H3Guard{a.ring_ovf, a.seq});
        }
        if (!(a.abl & 2)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
            __syncthreads();
        }
        if (tid == 0) __hip_atomic_fetch_add(cnt + (size_t)l * mtiles + mt, (unsigned)grp, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        w = __builtin_amdgcn_readfirstlane(s_claim[0]);
    }
}

template <int C, int BN, int WM, int TM, int NW, int VAR = 0, int HABL = 0>
static hipError_t launch_tower_t(const TowerArgs& a, hipStream_t st, int* grid_out)
{
    constexpr int lds = tower_lds_bytes<C, BN, WM, TM, NW, VAR>();
    static int grid = 0;
    if (grid == 0) {
        hipError_t e = hipFuncSetAttribute((const void*)conv_tower<C, BN, WM, TM, NW, VAR, HABL>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)conv_tower<C, BN, WM, TM, NW, VAR, HABL>,
                                                         64 * NW, lds);
        if (e != hipSuccess) return e;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        // the sc1-load hand-off (VAR 16) is valid at one workgroup per CU only: the
        // product refuses to launch it at any other residency (the study build runs the
        // round-2 two-per-CU form on purpose, key 31)
#ifndef AZG_AB_STUDIES
        if ((VAR & 16) && per_cu != 1) return hipErrorInvalidConfiguration;
#else
        if ((VAR & 16) && NW >= 16 && per_cu != 1) return hipErrorInvalidConfiguration;
#endif
        grid = max(1, per_cu) * cus;
    }
    if (grid_out) *grid_out = grid;
    hipLaunchKernelGGL((conv_tower<C, BN, WM, TM, NW, VAR, HABL>), dim3(grid), dim3(64 * NW), lds, st, a);
    return hipGetLastError();
}

int g_tower_ablation = 0;
int g_tower_var = 0;     // halo_tile VAR of the 128x64 C=128 tower (0 = product; 1..8, 12 A/B studies)
int g_tower_shape = 8;   // forced shape when g_tower_mode == 1: 5 = 64x64 (4 waves), 8 = 128x64 (8 waves),
                         // 10 = 128x128 (16 waves, one workgroup per CU; C = 128)

// [0] work counter, [1] error word, [4 ..) per-(layer, M tile) counters
size_t tower_sync_bytes(int nlayers, int M)
{
    const int mtiles = (M + 63) / 64;   // the smallest BM (64) has the most M tiles
    return ((size_t)(4 + nlayers * mtiles) * sizeof(unsigned) + 15) / 16 * 16;
}
// per-(layer, M tile) producer records (never cleared: tagged with the launch number)
size_t tower_prod_bytes(int nlayers, int M)
{
    const int mtiles = (M + 63) / 64;
    return (size_t)nlayers * mtiles * sizeof(uint4);
}

// Eval residual tower in one launch: NB blocks, conv1 X -> H (BN, ReLU), conv2
// H -> Y (BN, + X, ReLU), X <-> Y.  `act` are the three padded NHWC buffers
// (act[0] holds the stem output; the result ends in act[0] or act[2], returned in
// *result).  `sync` must hold tower_sync_bytes(2*NB, M) bytes.
int g_h3_tower_var = 1;   // key 20: the H3 tower body, 1 = board-keyed halo swizzle (VAR 99, default), 0 = row-keyed (98)
// key 19: split-fp16 (H3) eval residual convs: 2 (default) the 16x16x32 board tower at C = 128
// (pv_board16.hip; C = 256 as 1), 1 the 32x32x16 forms (pv_halo.h VAR bit 64), 0 fp32 MFMA
int g_tower_h3 = 2;

hipError_t launch_tower(int C, int NB, int shape, float* const act[3], const float* wpack, const float* scale,
                        const float* shift, const int* out_off, int M, const TowerSync& ts, hipStream_t st,
                        float** result, bool h3)
{
    if (2 * NB > kTowerMaxLayers) return hipErrorInvalidValue;
    const size_t act_bytes = (size_t)(M / PIX) * PADPIX * C * sizeof(float);
    if (act_bytes >= (size_t)INT32_MAX) return hipErrorInvalidValue;
    TowerArgs a{};
    a.nlayers = 2 * NB;
    a.M = M;
    a.act_bytes = (int)act_bytes;
    a.sync = ts.sync;
    a.ring = ts.ring;
    a.ring_ovf = ts.ring_ovf;
    a.diag = ts.diag;
    a.prod = (uint4*)ts.prod;
    a.seq = ts.seq;
    // microseconds -> 10-ns ticks, saturating
    a.limit = g_tower_wait_us >= 0xffffffffu / 100u ? 0xffffffffu : g_tower_wait_us * 100u;
    unsigned* sync = ts.sync;
    a.group = g_tower_group ? C / (shape == 8 || shape == 5 ? 64 : 128) : 1;
    if (shape == 12 && !h3) return hipErrorInvalidValue;   // h3_tile: split-fp16 only
#ifndef AZG_AB_STUDIES
    if (shape == 10 && C != 128) return hipErrorInvalidValue;   // 16-wave tile: C = 128 only (C = 256 spills)
#endif
    a.abl = g_tower_ablation;
    float* X = act[0];
    float* H = act[1];
    float* Y = act[2];
    for (int i = 0; i < NB; ++i) {
        TowerLayer& c1 = a.L[2 * i];
        c1 = TowerLayer{wpack + (size_t)(2 * i) * 9 * C * C, scale + out_off[2 * i], shift + out_off[2 * i], X,
                        nullptr, H};
        TowerLayer& c2 = a.L[2 * i + 1];
        c2 = TowerLayer{wpack + (size_t)(2 * i + 1) * 9 * C * C, scale + out_off[2 * i + 1],
                        shift + out_off[2 * i + 1], H, X, Y};
        float* t = X;
        X = Y;
        Y = t;
    }
    *result = X;
    hipError_t e = hipMemsetAsync(sync, 0, tower_sync_bytes(2 * NB, M), st);
    if (e != hipSuccess) return e;
    if (h3) {   // wpack / scale are the split-fp16 packs (pv_pack.hip pack_h3)
        // VAR 99 = H3 + buffer addressing + weights staged two chunks ahead (bit 2) + the
        // board-keyed halo swizzle (bit 1): with the fragment addresses built per tap (no
        // spills) 3.8-4.8 % faster than the row-keyed VAR 98, whose fragment reads conflict
        // at board-row ends (32 % of its LDS cycles; scripts/h3_tune_study.py,
        // profiles/r5_h3_study.md); bitwise equal to every other form.  Key 20 = 0: VAR 98.
        const bool vs = g_h3_tower_var == 1;
        // shape 12: h3_tile 128x128, 4 waves of 64x64 (VAR 355 = 99 | 256), bitwise equal
        if (shape == 12) {
            if (C == 128) return launch_tower_t<128, 128, 2, 2, 4, 355>(a, st, nullptr);
            if (C == 256) return launch_tower_t<256, 128, 2, 2, 4, 355>(a, st, nullptr);
            return hipErrorInvalidValue;
        }
        switch (C) {
            case 128:
                if (shape == 5) return vs ? launch_tower_t<128, 64, 2, 1, 4, 99>(a, st, nullptr)
                                          : launch_tower_t<128, 64, 2, 1, 4, 98>(a, st, nullptr);
                return vs ? launch_tower_t<128, 64, 4, 1, 8, 99>(a, st, nullptr)
                          : launch_tower_t<128, 64, 4, 1, 8, 98>(a, st, nullptr);
            case 256:
                if (shape == 5) return vs ? launch_tower_t<256, 64, 2, 1, 4, 99>(a, st, nullptr)
                                          : launch_tower_t<256, 64, 2, 1, 4, 98>(a, st, nullptr);
                return vs ? launch_tower_t<256, 64, 4, 1, 8, 99>(a, st, nullptr)
                          : launch_tower_t<256, 64, 4, 1, 8, 98>(a, st, nullptr);
            default: return hipErrorInvalidValue;
        }
    }
#ifdef AZG_AB_STUDIES
    // traffic ablations of the 128x64 tower (key 8 bits 4 / 8: no weight / no halo loads)
    if (shape == 8 && (a.abl & 12)) {
        const bool nw = a.abl & 4, nh = a.abl & 8;
        if (C == 256 && nw && nh) return launch_tower_t<256, 64, 4, 1, 8, 32, 3>(a, st, nullptr);
        if (C == 256 && nw) return launch_tower_t<256, 64, 4, 1, 8, 32, 1>(a, st, nullptr);
        if (C == 256 && nh) return launch_tower_t<256, 64, 4, 1, 8, 32, 2>(a, st, nullptr);
        if (C == 128 && nw && nh) return launch_tower_t<128, 64, 4, 1, 8, 32, 3>(a, st, nullptr);
        if (C == 128 && nw) return launch_tower_t<128, 64, 4, 1, 8, 32, 1>(a, st, nullptr);
        if (C == 128 && nh) return launch_tower_t<128, 64, 4, 1, 8, 32, 2>(a, st, nullptr);
    }
    if (g_tower_coh && (shape == 8 || shape == 5)) {   // study only: sc1 loads at 2-4 workgroups per CU
        if (C == 128 && shape == 8) return launch_tower_t<128, 64, 4, 1, 8, 16>(a, st, nullptr);
        if (C == 128) return launch_tower_t<128, 64, 2, 1, 4, 16>(a, st, nullptr);
    }
    if (C == 128 && shape == 9) {   // 128x128 tiles, 2 accumulators per wave, LDS-DMA staging (A/B study)
        if (g_tower_var == 5) return launch_tower_t<128, 128, 4, 1, 8, 5>(a, st, nullptr);
        return launch_tower_t<128, 128, 4, 1, 8, 4>(a, st, nullptr);
    }
    if (C == 128 && shape == 8 && g_tower_var != 0) {   // A/B variants (bitwise identical)
        if (g_tower_var == 3) return launch_tower_t<128, 64, 4, 1, 8, 3>(a, st, nullptr);
        if (g_tower_var == 1) return launch_tower_t<128, 64, 4, 1, 8, 1>(a, st, nullptr);
        if (g_tower_var == 2) return launch_tower_t<128, 64, 4, 1, 8, 2>(a, st, nullptr);
        if (g_tower_var == 4) return launch_tower_t<128, 64, 4, 1, 8, 4>(a, st, nullptr);
        if (g_tower_var == 5) return launch_tower_t<128, 64, 4, 1, 8, 5>(a, st, nullptr);
        if (g_tower_var == 8) return launch_tower_t<128, 64, 4, 1, 8, 8>(a, st, nullptr);
        if (g_tower_var == 6) return launch_tower_t<128, 64, 4, 1, 8, 6>(a, st, nullptr);
        if (g_tower_var == 7) return launch_tower_t<128, 64, 4, 1, 8, 7>(a, st, nullptr);
        if (g_tower_var == 12) return launch_tower_t<128, 64, 4, 1, 8, 12>(a, st, nullptr);
        if (g_tower_var == 14) return launch_tower_t<128, 64, 4, 1, 8, 33>(a, st, nullptr);
        if (g_tower_var == 15) return launch_tower_t<128, 64, 4, 1, 8, 34>(a, st, nullptr);
    }
    if (C == 256 && shape == 8 && g_tower_var == 2)   // weights staged two chunks ahead (VAR bit 2), C = 256
        return launch_tower_t<256, 64, 4, 1, 8, 34>(a, st, nullptr);
    if (C == 256 && shape == 8 && g_tower_var == 16)   // round-3 product body at C = 256 (VAR 32)
        return launch_tower_t<256, 64, 4, 1, 8, 32>(a, st, nullptr);
    if (C == 256 && shape == 5 && g_tower_var == 16)   // round-3 64x64 body at C = 256 (VAR 32)
        return launch_tower_t<256, 64, 2, 1, 4, 32>(a, st, nullptr);
    if (C == 256 && shape == 10) {   // 16-wave 128x128 tile at C = 256 (spills; traffic study)
        if (g_tower_var == 1) return launch_tower_t<256, 128, 4, 1, 16, 32>(a, st, nullptr);
        return launch_tower_t<256, 128, 4, 1, 16, 16>(a, st, nullptr);
    }
    if (C == 128 && shape == 5 && g_tower_var == 14) return launch_tower_t<128, 64, 2, 1, 4, 33>(a, st, nullptr);
    if (C == 128 && shape == 10 && g_tower_var == 1)   // 16-wave tile with the acquire instead of sc1 loads
        return launch_tower_t<128, 128, 4, 1, 16, 32>(a, st, nullptr);
    if (C == 128 && shape == 8 && g_tower_var == 13)   // round-2 acquire form: 64-bit pointer loads (VAR 0)
        return launch_tower_t<128, 64, 4, 1, 8, 0>(a, st, nullptr);
#endif
    switch (C) {
        case 64:
            if (shape == 8) return launch_tower_t<64, 64, 4, 1, 8, 32>(a, st, nullptr);
            return launch_tower_t<64, 64, 2, 1, 4, 32>(a, st, nullptr);
        case 128:
            if (shape == 10) return launch_tower_t<128, 128, 4, 1, 16, 16>(a, st, nullptr);
            if (shape == 8) return launch_tower_t<128, 64, 4, 1, 8, 32>(a, st, nullptr);
            return launch_tower_t<128, 64, 2, 1, 4, 32>(a, st, nullptr);
        case 256:
            // C = 256: halo rows keyed on the board position (VAR bit 1: conflict-free
            // fragment reads, unpadded epilogue tile), bitwise equal, scripts/gpu_r4o.sh:
            // 128x64 tile 90.0 vs 86.4 % of peak at B = 512, equal at 128 / 300 / 1024 /
            // 2048; 64x64 tile 79.4 vs 77.4 % at B = 300, 89.5 vs 88.2 % at 512, 55.4 vs
            // 56.4 % at 128.  At C = 128 the same body is slower (89.5 vs 91.2 % at B =
            // 3456), so C = 128 keeps VAR 32.
            if (shape == 8) return launch_tower_t<256, 64, 4, 1, 8, 33>(a, st, nullptr);
            return launch_tower_t<256, 64, 2, 1, 4, 33>(a, st, nullptr);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace azg
