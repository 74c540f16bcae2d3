// Persistent train backward: the whole residual-tower backward of one train step
// (reference network.py:12-25 through loss.backward() at network.py:224 -- per conv
// the BatchNorm backward apply, the data gradient with the next BN's backward sums and
// their finalize, the weight gradient and its split-K reduction) in ONE launch.
//
// Why: the two-stream schedule (tuning key 43 = 0) runs the dgrads on the caller's
// stream and the weight grads on a side stream; every cross-stream event record or wait
// costs the recording stream ~6 us (13 per step, traced), each dgrad is a 450-tile
// round on 512 slots, and every BN finalize (~6 us, one workgroup) and launch boundary
// sits on the critical path.  Here resident workgroups (two per CU, 8 waves) claim work
// items from one agent-scope counter in the order
//     group p = [A_p][D_p][W_p][R_{p-1}],  p = 0 .. nconv-1,  then R_{nconv-1}
// (BwdConv in pv_bwd_tower.h: A = BN-backward apply per 128-row tile, D = dgrad tile
// 128 x 64, W = weight-grad tile of one (pixel split, tap), R = 4096 slab-reduced
// weight-grad elements), so the weight-grad work of a conv fills the slots the next
// conv's dependency chain (last dgrad tile -> finalize -> apply -> dgrad) leaves idle.
// Waits (one lane polls relaxed agent-scope loads with s_sleep, bounded):
//   A_p: the finalize of its BN (both N tiles' last D_{p-1} workgroups; none for p = 0,
//        whose finalize ran before the launch);
//   D_p, W_p: every A_p item; W_p also every R_{p-3} item (three rotating slabs);
//   R_q: every W_q item.
// A tile only waits on items claimed before it, and a claimed item always runs on a
// resident workgroup, so the oldest unfinished item can always finish (deadlock-free,
// as the eval tower, pv_tower.hip).  A timed-out wait sets the error word and the
// sticky host-visible status (azg_pv_status) and the workgroup proceeds, so the grid
// always drains.
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", cdna_hip_programming.md Guideline 16):
// producer R1 -- every handed-off byte (dz, the residual gradient, dgrad outputs, BN
// partials and finalize results, slabs) is stored write-through (sc1), every storing
// wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, one lane adds to the counter
// with an agent-scope atomic; consumer -- one lane polls, ONE agent-scope acquire,
// vmcnt(0), a workgroup barrier, plain loads (the form valid at two workgroups per CU).
// Buffer reuse (WAR) is covered by the dependency chain: DH, gX, GR and the BN
// partials are rewritten only by items that (transitively) wait on every reader of the
// previous contents (the chain A_p -> D_p -> finalize -> A_{p+1} passes through all of
// them); dZ has one buffer per conv.
//
// Every item computes exactly what the stand-alone kernels of the two-stream schedule
// compute (the same tile bodies and per-element orders): the results are bitwise
// identical to it (tested, key 43).
#include "pv_bwd_tower.h"
#include "pv_wgrad.h"

namespace azg {

constexpr int kBwdThreads = 512;
constexpr int kBwdRed = 4096;          // weight-grad elements per R item (512 threads x 8)

template <int C>
constexpr int bwd_lds_bytes()
{
    constexpr int d = halo_lds_bytes<C, 64, 4, 1, 8, 0, PRO_NONE>();
    constexpr int w = WgNat<C>::LDS_BYTES;
    return (d > w ? d : w) + 16;
}

struct BwdArgs {
    const BwdConv* conv;
    int nconv;
    int M;
    int S;                 // weight-grad pixel splits
    unsigned* sync;
    unsigned* status;
    unsigned spin_limit;
    unsigned long long* trace;   // timing studies (AZG_BWD_TRACE): per item {claim, slot, t0, t1, t2}, or null
};

// poll *c >= target (one lane); false on timeout (error word + sticky status set)
__device__ __forceinline__ bool bwd_wait(const unsigned* c, unsigned target, const BwdArgs& a)
{
    unsigned spins = 0;
    while (a.spin_limit == 0 || __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++spins > a.spin_limit) {
            __hip_atomic_store(a.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// R1 publish of one item: every storing wave drains, barrier, one agent-scope add
__device__ __forceinline__ void bwd_publish(unsigned* c)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A item: BatchNorm backward apply of rows [m0, m0 + 128) (= bn_bwd_apply_kernel<C,
// GRES, true, MZ>, pv_train.hip: the same per-element expression, pv_wgrad.h bnbwd_elem)
template <int C>
__device__ __forceinline__ void bwd_apply_rows(const BwdConv& cv, int M, int m0)
{
    constexpr int F4 = C / 4;
    const int rows = min(TRAIN_BM, M - m0);
    const int total = rows * F4;
    const __amdgpu_buffer_rsrc_t rz = wt_rsrc(cv.dz, padded_bytes(M, C));
    const __amdgpu_buffer_rsrc_t rg = wt_rsrc(cv.gres ? cv.gres : cv.dz, padded_bytes(M, C));
    const bool mz = cv.act == nullptr;
#pragma unroll 2
    for (int i = threadIdx.x; i < total; i += kBwdThreads) {
        const int r = i / F4, c = (i - r * F4) * 4;
        const int o = pad_off(m0 + r, C) + c;
        const f32x4 gv = *(const f32x4*)(cv.g + o);
        const f32x4 zv = *(const f32x4*)(cv.z + o);
        f32x4 av;
        if (mz) {
            const f32x4 sc = *(const f32x4*)(cv.fscale + c), sh = *(const f32x4*)(cv.fshift + c);
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = fmaf(zv[q], sc[q], sh[q]);
        } else {
            av = *(const f32x4*)(cv.act + o);
        }
        const f32x4 mu = *(const f32x4*)(cv.mean + c);
        const f32x4 g_ = *(const f32x4*)(cv.gm + c);
        const f32x4 k_ = *(const f32x4*)(cv.kk + c);
        const f32x4 w_ = *(const f32x4*)(cv.iw + c);
        f32x4 out, dyv;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float dy;
            out[q] = bnbwd_elem(gv[q], av[q], zv[q], mu[q], g_[q], k_[q], w_[q], dy);
            dyv[q] = dy;
        }
        store4<true>(cv.dz, rz, o, out);
        if (cv.gres) store4<true>(cv.gres, rg, o, dyv);
    }
}

template <int C>
__global__ __launch_bounds__(kBwdThreads) __attribute__((amdgpu_waves_per_eu(4))) void train_bwd_tower(const BwdArgs a)
{
    using WG = WgNat<C>;
    constexpr int NTN = C / 64;                      // N tiles of a dgrad (64 channels each)
    constexpr int LDS_F = (bwd_lds_bytes<C>() - 16) / 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int* s_claim = (int*)(smem + LDS_F);

    const int tid = threadIdx.x;
    const int M = a.M;
    const int ntt = (M + TRAIN_BM - 1) / TRAIN_BM;
    const int nA = ntt, nD = ntt * NTN, nW = WG::TILES * a.S, nR = (9 * C * C + kBwdRed - 1) / kBwdRed;
    const int G0 = nA + nD + nW, G = G0 + nR;
    const int total = G0 + (a.nconv - 1) * G + nR;
    unsigned* work = a.sync;
    unsigned* cnt = a.sync + kBwdSyncHead;           // [p][4]: A done, W done, R done, fin

    if (tid == 0) s_claim[0] = (int)__hip_atomic_fetch_add(work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    int w = __builtin_amdgcn_readfirstlane(s_claim[0]);   // uniform: item decode in SGPRs
    while (w < total) {
        // decode: group p, offset in the group
        int p, off;
        if (w < G0) {
            p = 0;
            off = w;
        } else {
            const int q = (w - G0) / G;
            off = (w - G0) - q * G;
            p = q + 1;
        }
        // kind: 0 A, 1 D, 2 W, 3 R (of conv rq)
        int kind, idx, rq = 0;
        if (p == a.nconv) {
            kind = 3, idx = off, rq = a.nconv - 1;
        } else if (off < nA) {
            kind = 0, idx = off;
        } else if (off < nA + nD) {
            kind = 1, idx = off - nA;
        } else if (off < G0) {
            kind = 2, idx = off - nA - nD;
        } else {
            kind = 3, idx = off - G0, rq = p - 1;
        }
        __syncthreads();   // every wave has read s_claim and is done with the previous item's LDS
        unsigned long long t0 = 0, t1 = 0;
        if (a.trace && tid == 0) t0 = wall_clock64();
        if (tid == 0) {
            // the next claim now: its latency overlaps this item
            s_claim[0] = (int)__hip_atomic_fetch_add(work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool waited = false;
            if (kind == 0 && p > 0) {
                bwd_wait(cnt + 4 * p + 3, NTN, a);
                waited = true;
            } else if (kind == 1 || kind == 2) {
                bwd_wait(cnt + 4 * p + 0, (unsigned)nA, a);
                if (kind == 2 && p >= 3) bwd_wait(cnt + 4 * (p - 3) + 2, (unsigned)nR, a);
                waited = true;
            } else if (kind == 3) {
                bwd_wait(cnt + 4 * rq + 1, (unsigned)nW, a);
                waited = true;
            }
            if (waited) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (a.trace) t1 = wall_clock64();
        }
        __syncthreads();
        if (kind == 0) {
            const BwdConv& cv = a.conv[p];
            bwd_apply_rows<C>(cv, M, idx * TRAIN_BM);
            bwd_publish(cnt + 4 * p + 0);
        } else if (kind == 1) {
            // dgrad tile; its epilogue publishes the BN partials, and the last workgroup of
            // each N tile finalizes them and adds to fin of conv p + 1 (fx.done)
            const BwdConv& cv = a.conv[p];
            const int mt = idx / NTN, nt = idx - mt * NTN;
            halo_tile<C, 64, 4, 1, 8, EPI_OPTADD, true, 0, 32, XE_BNBWD, PRO_NONE>(
                cv.dz, cv.wd, nullptr, nullptr, cv.resid, cv.out, wt_rsrc(cv.out, padded_bytes(M, C)), M,
                mt * TRAIN_BM, nt * 64, smem, cv.ex, ProX{}, cv.fx);
        } else if (kind == 2) {
            const BwdConv& cv = a.conv[p];
            const int split = idx / WG::TILES;
            int t = idx - split * WG::TILES;
            const int tap = t / (WG::NT * WG::NT);
            t -= tap * WG::NT * WG::NT;
            wgrad_nat_tile<C, true, WG::NWV>(cv.dz, cv.wx, cv.slab, M, a.S, split, tap, (t / WG::NT) * WG::BT,
                                             (t % WG::NT) * WG::BT, smem);
            bwd_publish(cnt + 4 * p + 1);
        } else {
            const BwdConv& cv = a.conv[rq];
            wgrad_reduce_elems<kBwdRed / kBwdThreads>(cv.slab, cv.dw, C, a.S, idx * kBwdRed + tid, kBwdThreads);
            bwd_publish(cnt + 4 * rq + 2);
        }
        if (a.trace && tid == 0) {
            unsigned long long* tr = a.trace + (size_t)w * 5;
            tr[0] = (unsigned long long)w;
            tr[1] = blockIdx.x;
            tr[2] = t0;
            tr[3] = t1;
            tr[4] = wall_clock64();
        }
        w = __builtin_amdgcn_readfirstlane(s_claim[0]);
    }
    // the last workgroup out re-arms every counter for the next launch
    if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            const int nw = bwd_sync_words(a.nconv);
            for (int i = 0; i < nw; ++i) __hip_atomic_store(a.sync + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int C>
static hipError_t launch_bwd_tower_t(const BwdArgs& a, hipStream_t st)
{
    constexpr int lds = bwd_lds_bytes<C>();
    static int grid = 0;
    if (grid == 0) {
        hipError_t e = hipFuncSetAttribute((const void*)train_bwd_tower<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           lds);
        if (e != hipSuccess) return e;
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)train_bwd_tower<C>, kBwdThreads, lds);
        if (e != hipSuccess) return e;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        grid = max(1, per_cu) * cus;
    }
    hipLaunchKernelGGL((train_bwd_tower<C>), dim3(grid), dim3(kBwdThreads), lds, st, a);
    return hipGetLastError();
}

int bwd_tower_items(int C, int nconv, int M, int S)
{
    const int ntt = (M + TRAIN_BM - 1) / TRAIN_BM, nt = C < 128 ? 1 : C / 128;
    const int G0 = ntt + ntt * (C / 64) + 9 * nt * nt * S, nR = (9 * C * C + kBwdRed - 1) / kBwdRed;
    return G0 + (nconv - 1) * (G0 + nR) + nR;
}

hipError_t launch_bwd_tower(int C, const BwdConv* desc, int nconv, int M, int S, unsigned* sync, unsigned* status,
                            hipStream_t st, unsigned long long* trace)
{
    if (nconv < 1 || S < 1 || M < 1) return hipErrorInvalidValue;
    BwdArgs a{desc, nconv, M, S, sync, status, g_tower_spin_limit, trace};
    switch (C) {
        case 64: return launch_bwd_tower_t<64>(a, st);
        case 128: return launch_bwd_tower_t<128>(a, st);
        case 256: return launch_bwd_tower_t<256>(a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace azg
