// Stand-alone timing lab for the conv weight-gradient GEMM (study tool, not product):
//   dW[tap][co][ci] = sum_m dz[m][co] * x[m + off(tap)][ci]   (6x128 net, B = 128)
// Compares the product kernel (pv_wgrad.hip conv3x3_wgrad_t + wgrad_reduce) with
// lab variants: 8-wave workgroups, a balanced (tap, chunk) unit split per XCD band,
// ablations (no slab stores / no global loads / no barriers; timing only).
// Checked against an fp64 reference on the GPU.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/wgrad_lab.hip -o scripts/wgrad_lab
#include "../alphazero-gomoku_amd/csrc/pv_wgrad.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace azg {
int g_train_wt = 7;
}
using namespace azg;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

// ---- lab kernel ----------------------------------------------------------
// NWV = 4: waves 2 (co) x 2 (ci), 64x64 each (2x2 accumulators);
// NWV = 8: waves 2 (co) x 4 (ci), 64x32 each (2x1 accumulators).
// BAL: workgroup w of XCD band b covers units [u0, u1) of the band's 9 x nchunk
// (tap-major) units; accumulators are flushed to slab segment (w, seg) at a tap change.
// ABL: 1 no slab stores, 2 no global loads, 4 no barriers (timing only).
constexpr int LC = 128;
template <int NWV, int ABL, bool BAL, bool WT>
__global__ __launch_bounds__(64 * NWV, 2) void wg_lab(const float* __restrict__ dz, const float* __restrict__ x,
                                                      float* __restrict__ slab, int M, int rps, int bandch)
{
    constexpr int C = LC, BT = 128, BK = 32, LDT = BK + 4;
    constexpr int NT = 64 * NWV;
    constexpr int WCI = NWV == 4 ? 2 : 4;           // waves along ci
    constexpr int TI = 2, TJ = NWV == 4 ? 2 : 1;    // accumulators per wave
    constexpr int W_CO = 64, W_CI = BT / WCI;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;
    float* Bs = smem + 2 * BT * LDT;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WCI, wn = wid % WCI;
    const int r32 = lane & 31, h = lane >> 5;
    const int nchunk_all = (M + BK - 1) / BK;

    // work: list of (tap, kc range) segments
    int seg_tap[2], seg_k0[2], seg_k1[2], nseg = 0;
    int slab_base;
    if (BAL) {
        const int xcd = blockIdx.x & 7, wl = blockIdx.x >> 3, G8 = gridDim.x >> 3;
        const int c0 = xcd * bandch, c1 = min(nchunk_all, c0 + bandch), nb = max(0, c1 - c0);
        const long U = 9L * nb;
        const int u0 = (int)(U * wl / G8), u1 = (int)(U * (wl + 1) / G8);
        int u = u0;
        while (u < u1 && nseg < 2) {
            const int tap = u / nb, k = u - tap * nb;
            const int e = min(u1, (tap + 1) * nb);
            seg_tap[nseg] = tap;
            seg_k0[nseg] = c0 + k;
            seg_k1[nseg] = c0 + k + (e - u);
            ++nseg;
            u = e;
        }
        slab_base = blockIdx.x * 2;
    } else {
        constexpr int TILES = 9;
        const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
        const int split = (k / TILES) * 8 + xcd;
        const int tap = k % TILES;
        const int mbeg = split * rps, mend = min(M, mbeg + rps);
        seg_tap[0] = tap;
        seg_k0[0] = 0;
        seg_k1[0] = (mend - mbeg + BK - 1) / BK;
        nseg = 1;
        slab_base = split * 9 + tap;
        // chunk index relative to mbeg below
    }
    const int mbase = BAL ? 0 : ((((blockIdx.x >> 3) / 9) * 8 + (blockIdx.x & 7)) * rps);
    const int mlim = BAL ? M : min(M, mbase + rps);

    // staging: 4x4 (pixel x channel) blocks; NWV=4: each thread stages one block of
    // both operands; NWV=8: threads 0-255 stage dz, 256-511 stage x
    constexpr int NBLK = (BT / 4) * (BK / 4);   // 256
    const int sid = tid % NBLK;
    const int pb = sid % (BK / 4), cb = sid / (BK / 4);
    const bool do_a = NWV == 4 || tid < NBLK;
    const bool do_b = NWV == 4 || tid >= NBLK;
    f32x4 ra[4], rb[4];

    f32x16 acc[TI][TJ];
    for (int s = 0; s < nseg; ++s) {
        const int tap = seg_tap[s];
        const int ky = tap / 3, kx = tap - ky * 3;
        const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
        const int k0 = seg_k0[s], k1 = seg_k1[s];
        auto gload = [&](int kc) {
            if (ABL & 2) return;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = mbase + kc * BK + 4 * pb + i;
                if (m < mlim) {
                    const int po = pad_off(m, C);
                    if (do_a) ra[i] = *(const f32x4*)(dz + po + 4 * cb);
                    if (do_b) rb[i] = *(const f32x4*)(x + po + toff + 4 * cb);
                } else {
                    ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                    rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
        };
        auto lstore = [&](int buf) {
            float* a = As + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
            float* b = Bs + buf * BT * LDT + (4 * cb) * LDT + 4 * pb;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (do_a) *(f32x4*)(a + j * LDT) = f32x4{ra[0][j], ra[1][j], ra[2][j], ra[3][j]};
                if (do_b) *(f32x4*)(b + j * LDT) = f32x4{rb[0][j], rb[1][j], rb[2][j], rb[3][j]};
            }
        };
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        if (k1 > k0) {
            gload(k0);
            lstore(0);
        }
        __syncthreads();
        for (int kc = k0; kc < k1; ++kc) {
            const int cur = (kc - k0) & 1;
            if (kc + 1 < k1) gload(kc + 1);
            __builtin_amdgcn_sched_barrier(0);
            const float* Ab = As + cur * BT * LDT + (wm * W_CO + r32) * LDT + h * (BK / 2);
            const float* Bb = Bs + cur * BT * LDT + (wn * W_CI + r32) * LDT + h * (BK / 2);
#pragma unroll
            for (int q = 0; q < BK / 8; ++q) {
                f32x4 a[TI], b[TJ];
#pragma unroll
                for (int i = 0; i < TI; ++i) a[i] = *(const f32x4*)(Ab + i * 32 * LDT + 4 * q);
#pragma unroll
                for (int j = 0; j < TJ; ++j) b[j] = *(const f32x4*)(Bb + j * 32 * LDT + 4 * q);
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                    for (int i = 0; i < TI; ++i)
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s4], b[j][s4], acc[i][j], 0, 0, 0);
            }
            if (kc + 1 < k1) lstore(cur ^ 1);
            if (!(ABL & 4)) __syncthreads();
        }
        float* out = slab + (size_t)(slab_base + s) * C * C;
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, (size_t)C * C * sizeof(float));
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = wm * W_CO + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int ci = wn * W_CI + j * 32 + r32;
                    if (!(ABL & 1) || acc[i][j][r] == 1234.5f) store1<WT>(out, rs, co * C + ci, acc[i][j][r]);
                }
        __syncthreads();
    }
}

// BAL reduce: dW[co][ci][tap] = sum over (xcd band, workgroup) segments of tap, fixed order
__global__ void wg_lab_reduce(const float* __restrict__ slab, float* __restrict__ dw, int M, int G, int bandch)
{
    constexpr int C = LC;
    const int nchunk_all = (M + 31) / 32;
    const int G8 = G / 8;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < 9 * C * C; idx += gridDim.x * blockDim.x) {
        const int tap = idx / (C * C), rem = idx - tap * C * C;
        float acc = 0.f;
        for (int xcd = 0; xcd < 8; ++xcd) {
            const int c0 = xcd * bandch, c1 = min(nchunk_all, c0 + bandch), nb = max(0, c1 - c0);
            if (!nb) continue;
            const long U = 9L * nb;
            const long ulo = (long)tap * nb, uhi = ulo + nb;
            // workgroups whose [u0, u1) meets [ulo, uhi)
            for (int wl = 0; wl < G8; ++wl) {
                const long u0 = U * wl / G8, u1 = U * (wl + 1) / G8;
                if (u1 <= ulo || u0 >= uhi || u1 == u0) continue;
                const int seg = (u0 >= ulo) ? 0 : 1;
                acc += slab[((size_t)(wl * 8 + xcd) * 2 + seg) * C * C + rem];
            }
        }
        dw[rem * 9 + tap] = acc;
    }
}

__global__ void wg_ref(const float* dz, const float* x, double* dw, int M)
{
    constexpr int C = LC;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= 9 * C * C) return;
    const int tap = idx / (C * C), rem = idx - tap * C * C, co = rem / C, ci = rem % C;
    const int ky = tap / 3, kx = tap % 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    double s = 0;
    for (int m = 0; m < M; ++m) {
        const int po = pad_off(m, C);
        s += (double)dz[po + co] * (double)x[po + toff + ci];
    }
    dw[rem * 9 + tap] = s;
}

__global__ void fill_padded(float* t, int B, unsigned seed)
{
    constexpr int C = LC;
    const long n = (long)B * PADPIX * C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long pix = i / C;
        const int pp = pix % PADPIX, yy = pp / PADW, xx = pp % PADW;
        unsigned hsh = (unsigned)i * 2654435761u ^ seed;
        hsh ^= hsh >> 13;
        hsh *= 0x5bd1e995u;
        hsh ^= hsh >> 15;
        const float v = ((hsh & 0xffff) / 65536.f) - 0.5f;
        t[i] = (yy >= 1 && yy <= BOARD && xx >= 1 && xx <= BOARD) ? v : 0.f;
    }
}


// NAT: natural [pixel][channel] LDS rows filled by global_load_lds (no staging
// registers, no transposition, no ds_write); 16-B chunk j of row p sits at slot
// j ^ 8*((p >> 4) & 1), so the b32 fragment reads (lanes 0-31: pixel s, lanes 32-63:
// pixel s + 16, 32 consecutive channels) are conflict-free.  Rows past the split
// read the zero halo row (padded pixel 0).
template <int ABL, int MODE = 0, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 2) void wg_nat(const float* __restrict__ dz, const float* __restrict__ x,
                                                 float* __restrict__ slab, int M, int rps, int bandch)
{
    constexpr int C = LC, BK = 32;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                 // [2][BK][C]
    float* Bs = smem + 2 * BK * C;    // [2][BK][C]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int WCI = NWV / 2, TJ = NWV == 4 ? 2 : 1, WW = 128 / WCI;
    const int wm = wid / WCI, wn = wid % WCI;
    const int r32 = lane & 31, h = lane >> 5;
    // segments (tap, chunk range [k0, k1) of 32-pixel chunks from pixel 0)
    int seg_tap[2], seg_k0[2], seg_k1[2], nseg = 0, slab_base;
    const int nchunk_all = (M + BK - 1) / BK;
    if (MODE == 2) {   // balanced (tap, chunk) units per XCD band
        const int xcd = blockIdx.x & 7, wl = blockIdx.x >> 3, G8 = gridDim.x >> 3;
        const int c0 = xcd * bandch, c1 = min(nchunk_all, c0 + bandch), nb = max(0, c1 - c0);
        const long U = 9L * nb;
        const int u0 = (int)(U * wl / G8), u1 = (int)(U * (wl + 1) / G8);
        int u = u0;
        while (u < u1 && nseg < 2) {
            const int tap = u / nb, k = u - tap * nb;
            const int e = min(u1, (tap + 1) * nb);
            seg_tap[nseg] = tap;
            seg_k0[nseg] = c0 + k;
            seg_k1[nseg] = c0 + k + (e - u);
            ++nseg;
            u = e;
        }
        slab_base = blockIdx.x * 2;
    } else {
        const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
        const int S = gridDim.x / 9;
        const int split = (k / 9) * 8 + xcd;
        seg_tap[0] = k % 9;
        if (MODE == 1) {   // whole chunks: split s gets chunks [s*N/S, (s+1)*N/S)
            seg_k0[0] = (int)((long)split * nchunk_all / S);
            seg_k1[0] = (int)((long)(split + 1) * nchunk_all / S);
        } else {           // product: rps rows per split (last chunk partial)
            seg_k0[0] = 0;
            seg_k1[0] = 0;
        }
        nseg = 1;
        slab_base = split * 9 + seg_tap[0];
    }
    const int xsplit = ((blockIdx.x >> 3) / 9) * 8 + (blockIdx.x & 7);
    const int mbeg = MODE == 0 ? xsplit * rps : 0;
    const int mend = MODE == 0 ? min(M, mbeg + rps) : M;
    if (MODE == 0) seg_k1[0] = (mend - mbeg + BK - 1) / BK;
    auto glds = [](const float* src, float* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ca = wm * 64 + i * 32 + r32, cbb = wn * WW + (i % TJ) * 32 + r32;
        aoff[i] = 16 * h * C + (((ca >> 2) ^ (h << 3)) << 2) + (ca & 3);
        boff[i] = 16 * h * C + (((cbb >> 2) ^ (h << 3)) << 2) + (cbb & 3);
    }
  for (int sg = 0; sg < nseg; ++sg) {
    const int tap = seg_tap[sg];
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    const int k0 = seg_k0[sg], nch = seg_k1[sg] - k0;
    // wave wid loads pixel rows RW*wid .. of each operand (RW/2 instructions each)
    constexpr int RW = 32 / NWV;
    auto issue = [&](int kc, int buf) {
        if (ABL & 2) return;
#pragma unroll
        for (int i = 0; i < RW / 2; ++i) {
            const int p = RW * wid + 2 * i + h;
            const int m = mbeg + (k0 + kc) * BK + p;
            const int j = r32 ^ (((p >> 4) & 1) << 3);
            const int po = m < mend ? pad_off(m, C) : 0;
            const int pox = m < mend ? po + toff : 0;
            glds(dz + po + 4 * j, As + buf * BK * C + (RW * wid + 2 * i) * C);
            glds(x + pox + 4 * j, Bs + buf * BK * C + (RW * wid + 2 * i) * C);
        }
    };
    f32x16 acc[2][TJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if (nch > 0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kc = 0; kc < nch; ++kc) {
        const int cur = kc & 1;
        if (kc + 1 < nch) issue(kc + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        const float* Ab = As + cur * BK * C;
        const float* Bb = Bs + cur * BK * C;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            float a[2], b[TJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = Ab[s * C + aoff[i]];
#pragma unroll
            for (int j = 0; j < TJ; ++j) b[j] = Bb[s * C + boff[j]];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!(ABL & 4)) __syncthreads();
    }
    float* out = slab + (size_t)(slab_base + sg) * C * C;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(out, (size_t)C * C * sizeof(float));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int ci = wn * WW + j * 32 + r32;
                if (!(ABL & 1) || acc[i][j][r] == 1234.5f) store1<true>(out, rs, co * C + ci, acc[i][j][r]);
            }
    __syncthreads();
  }
}

template <int ABL, int MODE = 0, int NWV = 4>
static float run_nat(const float* dz, const float* x, float* slab, float* dw, int M, int iters, float* ms_kernel)
{
    constexpr int lds = 2 * 2 * 32 * 128 * 4;
    CK(hipFuncSetAttribute((const void*)wg_nat<ABL, MODE, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int S = wgrad_splits(LC, M), rps = 0;
    const int bandch = ((M + 31) / 32 + 7) / 8;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    float tk = 0, tt = 0;
    for (int it = -2; it < iters; ++it) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((wg_nat<ABL, MODE, NWV>), dim3(MODE == 2 ? 512 : S * 9), dim3(64 * NWV), lds, 0, dz, x, slab, M, rps,
                           bandch);
        CK(hipEventRecord(e1, 0));
        if (MODE == 2)
            hipLaunchKernelGGL(wg_lab_reduce, dim3(576), dim3(256), 0, 0, slab, dw, M, 512, bandch);
        else
            hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((9 * LC * LC + 255) / 256), dim3(256), 0, 0, slab, dw, LC, S);
        CK(hipEventRecord(e2, 0));
        CK(hipEventSynchronize(e2));
        float a, b;
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventElapsedTime(&b, e0, e2));
        if (it >= 0) {
            tk += a;
            tt += b;
        }
    }
    *ms_kernel = tk / iters;
    return tt / iters;
}

template <int NWV, int ABL, bool BAL, bool WT>
static float run_lab(const float* dz, const float* x, float* slab, float* dw, int M, int iters, bool reduce,
                     float* ms_kernel)
{
    constexpr int lds = 2 * 2 * 128 * 36 * 4;
    CK(hipFuncSetAttribute((const void*)wg_lab<NWV, ABL, BAL, WT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int G = 512;
    const int nch = (M + 31) / 32;
    const int bandch = (nch + 7) / 8;
    const int S = wgrad_splits(LC, M), rps = 0;
    const int grid = BAL ? G : S * 9;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    float tk = 0, tt = 0;
    for (int it = -2; it < iters; ++it) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((wg_lab<NWV, ABL, BAL, WT>), dim3(grid), dim3(64 * NWV), lds, 0, dz, x, slab, M, rps, bandch);
        CK(hipEventRecord(e1, 0));
        if (reduce) {
            if (BAL)
                hipLaunchKernelGGL(wg_lab_reduce, dim3(576), dim3(256), 0, 0, slab, dw, M, G, bandch);
            else
                hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((9 * LC * LC + 255) / 256), dim3(256), 0, 0, slab, dw,
                                   LC, S);
        }
        CK(hipEventRecord(e2, 0));
        CK(hipEventSynchronize(e2));
        float a, b;
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventElapsedTime(&b, e0, e2));
        if (it >= 0) {
            tk += a;
            tt += b;
        }
    }
    *ms_kernel = tk / iters;
    return tt / iters;
}

static double check(const float* dw_d, const std::vector<double>& ref)
{
    std::vector<float> h(ref.size());
    CK(hipMemcpy(h.data(), dw_d, h.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, er = 0;
    for (size_t i = 0; i < h.size(); ++i) {
        mx = fmax(mx, fabs(ref[i]));
        er = fmax(er, fabs(h[i] - ref[i]));
    }
    return er / mx;
}

int main(int argc, char** argv)
{
    const int B = argc > 1 ? atoi(argv[1]) : 128;
    const int iters = argc > 2 ? atoi(argv[2]) : 50;
    const int M = B * PIX;
    const size_t n = (size_t)B * PADPIX * LC;
    float *dz, *x, *slab, *dw;
    double* dref;
    CK(hipMalloc(&dz, n * 4));
    CK(hipMalloc(&x, n * 4));
    CK(hipMalloc(&slab, (size_t)1024 * 2 * LC * LC * 4));
    CK(hipMalloc(&dw, 9 * LC * LC * 4));
    CK(hipMalloc(&dref, 9 * LC * LC * 8));
    hipLaunchKernelGGL(fill_padded, dim3(2048), dim3(256), 0, 0, dz, B, 1u);
    hipLaunchKernelGGL(fill_padded, dim3(2048), dim3(256), 0, 0, x, B, 7u);
    hipLaunchKernelGGL(wg_ref, dim3((9 * LC * LC + 255) / 256), dim3(256), 0, 0, dz, x, dref, M);
    CK(hipDeviceSynchronize());
    std::vector<double> ref(9 * LC * LC);
    CK(hipMemcpy(ref.data(), dref, ref.size() * 8, hipMemcpyDeviceToHost));
    const double flop = 2.0 * M * 9 * LC * LC;
    const int S = wgrad_splits(LC, M), rps = 0;
    printf("B=%d M=%d product split S=%d rps=%d (grid %d)\n", B, M, S, rps, S * 9);

    // product path
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float t = 0;
        for (int it = -2; it < iters; ++it) {
            CK(hipEventRecord(e0, 0));
            CK(launch_wgrad(LC, dz, x, slab, dw, M, S, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float a;
            CK(hipEventElapsedTime(&a, e0, e1));
            if (it >= 0) t += a;
        }
        t /= iters;
        printf("%-34s total %7.1f us  (%.1f%% of 157.3 TF)  err %.2e\n", "product (kernel+reduce)", t * 1e3,
               flop / (t * 1e-3) / 157.3e12 * 100, check(dw, ref));
    }
#define LAB(NWV, ABL, BAL, WT, NAME)                                                                           \
    {                                                                                                          \
        float tk;                                                                                              \
        float t = run_lab<NWV, ABL, BAL, WT>(dz, x, slab, dw, M, iters, true, &tk);                            \
        printf("%-34s total %7.1f us kernel %7.1f us (%.1f%%)  err %.2e\n", NAME, t * 1e3, tk * 1e3,           \
               flop / (tk * 1e-3) / 157.3e12 * 100, ABL ? 0.0 : check(dw, ref));                             \
    }
    LAB(4, 0, false, true, "lab 4w split (=product)");
    LAB(4, 1, false, true, "lab 4w split, no slab store");
    LAB(4, 2, false, true, "lab 4w split, no global loads");
    LAB(4, 4, false, true, "lab 4w split, no barriers");
    LAB(4, 0, false, false, "lab 4w split, slab write-back");
    LAB(8, 0, false, true, "lab 8w split");
    LAB(8, 1, false, true, "lab 8w split, no slab store");
    LAB(4, 0, true, true, "lab 4w balanced");
    LAB(4, 1, true, true, "lab 4w balanced, no slab store");
    LAB(8, 0, true, true, "lab 8w balanced");
    LAB(8, 0, true, false, "lab 8w balanced, write-back");
    LAB(8, 1, true, true, "lab 8w balanced, no slab store");
    LAB(8, 2, true, true, "lab 8w balanced, no global loads");

#define NAT(ABL, NAME, ...)                                                                                    \
    {                                                                                                          \
        float tk;                                                                                              \
        float t = run_nat<ABL, ##__VA_ARGS__>(dz, x, slab, dw, M, iters, &tk);                                             \
        printf("%-34s total %7.1f us kernel %7.1f us (%.1f%%)  err %.2e\n", NAME, t * 1e3, tk * 1e3,           \
               flop / (tk * 1e-3) / 157.3e12 * 100, ABL ? 0.0 : check(dw, ref));                             \
    }
    NAT(0, "nat glds b32");
    NAT(1, "nat glds b32, no slab store");
    NAT(2, "nat glds b32, no global loads");
    NAT(4, "nat glds b32, no barriers");
    NAT(0, "nat exact chunks", 1);
    NAT(6, "nat exact, no loads, no barriers", 1);
    NAT(0, "nat exact 8 waves", 1, 8);
    NAT(2, "nat exact 8 waves, no loads", 1, 8);
    NAT(0, "nat balanced units", 2);
    NAT(1, "nat balanced, no slab store", 2);
    NAT(2, "nat balanced, no global loads", 2);
    {
        g_wgrad_kernel = 2;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float t = 0;
        for (int it = -2; it < iters; ++it) {
            CK(hipEventRecord(e0, 0));
            CK(launch_wgrad(LC, dz, x, slab, dw, M, S, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float a;
            CK(hipEventElapsedTime(&a, e0, e1));
            if (it >= 0) t += a;
        }
        t /= iters;
        g_wgrad_kernel = 1;
        printf("%-34s total %7.1f us  err %.2e\n", "product PF2 (kernel+reduce)", t * 1e3, check(dw, ref));
    }
    return 0;
}
