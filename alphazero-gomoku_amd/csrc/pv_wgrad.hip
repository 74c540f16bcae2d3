// Weight gradient of the 3x3 convolution (autograd of network.py:12,14 conv2d):
//   dW[co][ci][tap] = sum_m dz[m][co] * X[m + off(tap)][ci]
// as an fp32-MFMA GEMM with co x ci outputs per tap and K = pixels of the batch,
// split over pixel slabs (split-K) so the grid fills the chip: every workgroup
// writes its 128x128 (64x64 at C=64) partial tile to a slab; wgrad_reduce sums
// the slabs in a fixed order (bitwise reproducible) into torch's [Cout][Cin][3][3].
//
// Operand staging keeps the natural NHWC rows ([32 pixels][channels]) in LDS;
// MFMA fragments are read with ds_read_b32 (lanes 0-31 read 32 consecutive
// channels of one pixel: conflict-free).  Rows past M load zeros.
#include "pv_internal.h"

namespace azg {

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
    int M, int rows_per_split)
{
    using T = WgTile<C, BK_>;
    constexpr int BT = T::BT, BK = T::BK, LD = T::LD, W = T::W, TT = T::T, LDF4 = T::LDF4, NT = T::NT;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                 // [2][BK][LD]  dz rows
    float* Bs = smem + 2 * BK * LD;   // [2][BK][LD]  x rows

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int split = blockIdx.x;
    int t = blockIdx.y;
    const int tap = t / (NT * NT);
    t -= tap * NT * NT;
    const int co0 = (t / NT) * BT, ci0 = (t % NT) * BT;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ((ky - 1) * PADW + (kx - 1)) * C;
    const int mbeg = split * rows_per_split;
    const int mend = min(M, mbeg + rows_per_split);
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

// dW (torch layout [co][ci][3][3]) = sum over slabs, fixed order: four interleaved
// partial sums (slabs k = 0,1,2,3 mod 4: independent loads in flight) combined as
// ((p0 + p1) + (p2 + p3)).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                           int C, int S)
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

template <int C, int BK = 32>
static hipError_t launch_wgrad_t(const float* dz, const float* x, float* slab, float* dw, int M, int S, int rps,
                                 hipStream_t st)
{
    using T = WgTile<C, BK>;
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_mfma<C, BK>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS_BYTES);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    dim3 grid(S, 9 * T::NT * T::NT);
    hipLaunchKernelGGL((conv3x3_wgrad_mfma<C, BK>), grid, dim3(256), T::LDS_BYTES, st, dz, x, slab, M, rps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int total = 9 * C * C;
    int nb = (total + 255) / 256;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nb), dim3(256), 0, st, slab, dw, C, S);
    return hipGetLastError();
}

// Rows per split (multiple of 32, >= 256): minimise rounds-of-workgroups x chunks
// per workgroup + the slab reduction (S slabs of 9*C*C floats re-read once).  The
// old fixed 512 gave 57 x 9 = 513 workgroups at B = 128 on 512 slots: one extra round.
int g_wgrad_bk = 32;   // pixels per K chunk of the wgrad tile (32 default; 16 = A/B study)

int wgrad_rows_per_split(int C, int M)
{
    const int bt = C < 128 ? C : 128;
    const int tiles = 9 * (C / bt) * (C / bt);
    const int lds = 2 * 2 * g_wgrad_bk * (bt + 4) * 4;
    const int slots = 256 * (160 * 1024 / lds);
    const double chunk_us = 5.4 * (bt / 128.0) * (bt / 128.0) * (160.0 * 1024 / lds) / 2.0;
    const double red_us = 9.0 * C * C * 4 / 4.0e6;     // one slab at ~4 TB/s
    int best = 512;
    double best_cost = 1e30;
    for (int rps = 256; rps <= 4096; rps += 32) {
        const int S = (M + rps - 1) / rps;
        const int rounds = (S * tiles + slots - 1) / slots;
        const double cost = rounds * (rps / 32) * chunk_us + S * red_us;
        if (cost < best_cost - 1e-9) { best_cost = cost; best = rps; }
        if (S == 1) break;
    }
    return best;
}

// slab must hold S*9*C*C floats, S = ceil(M / rps).
hipError_t launch_wgrad(int C, const float* dz, const float* x, float* slab, float* dw, int M, int S, int rps,
                        hipStream_t st)
{
    switch (C) {
        case 64: return launch_wgrad_t<64>(dz, x, slab, dw, M, S, rps, st);
        case 128:
            if (g_wgrad_bk == 16) return launch_wgrad_t<128, 16>(dz, x, slab, dw, M, S, rps, st);
            return launch_wgrad_t<128>(dz, x, slab, dw, M, S, rps, st);
        case 256: return launch_wgrad_t<256>(dz, x, slab, dw, M, S, rps, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace azg
