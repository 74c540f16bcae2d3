// Weight gradient of the 3x3 convolution (autograd of network.py:12,14 conv2d):
//   dW[co][ci][tap] = sum_m dz[m][co] * X[m + off(tap)][ci]
// as an fp32-MFMA GEMM with co x ci outputs per tap and K = pixels of the batch,
// split over pixel slabs (split-K) so the grid fills the chip: every workgroup
// writes its 128x128 (64x64 at C=64) partial tile to a slab; wgrad_reduce sums
// the slabs in a fixed order (bitwise reproducible) into torch's [Cout][Cin][3][3].
// The tile bodies and the reduction orders live in pv_wgrad.h; these are the launches
// of the train step's two-stream backward schedule.
#include "pv_internal.h"
#include "pv_wgrad.h"

namespace azg {

// One tile per workgroup, 4 waves (2 x 2 of (BT/2)^2).  XCD-aware order
// (cdna_hip_programming.md T1; speed only): blocks b and b+8 share an XCD, so every
// tile of one pixel split is given to the same block label b % 8 -- the split's dz
// rows and (tap-shifted) x rows are fetched into that XCD's L2 once and served to all
// of its tiles.  gridDim.x = S * TILES with S % 8 == 0.  Measured at 6x128, B = 128
// (scripts/wgrad_lab.hip): 74.0 us vs 89.2 for a K-contiguous register-staged kernel.
template <int C>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_nat(const float* __restrict__ dz, const float* __restrict__ x,
                                                            float* __restrict__ slab, int M, int S)
{
    using W = WgNat<C>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int split = (k / W::TILES) * 8 + xcd;
    int t = k % W::TILES;
    const int tap = t / (W::NT * W::NT);
    t -= tap * W::NT * W::NT;
    wgrad_nat_tile<C, true, 4>(dz, x, slab, M, S, split, tap, (t / W::NT) * W::BT, (t % W::NT) * W::BT, smem);
}

// dW = the S slabs summed in a fixed order (pv_wgrad.h wgrad_reduce_vec4: the per-element
// order of wgrad_reduce_elems), one float4 run per thread.  In the step this pass shares
// the chip with a dgrad; a quarter of the load instructions of the 4-scalar form made the
// step 21 us faster (2.843-2.848 vs 2.864-2.872 ms, scripts/gpu_r4l.sh; two float4 per
// thread: 2.875-2.882), bitwise equal.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                           int C, int S)
{
    wgrad_reduce_vec4<1>(slab, dw, C, S, blockIdx.x * 256 + threadIdx.x, 256);
}

// Round 5 (key 48 = 1, default): the v2 tile (pv_wgrad.h wgrad_nat_tile2 -- row table,
// buffer LDS-DMA, MFMA-layout slabs), bitwise equal to v1's slabs summed in v1's order.
int g_wgrad_variant = 1;

template <int C>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_nat2(const float* __restrict__ dz, const float* __restrict__ x,
                                                             const int* __restrict__ rowtab, float* __restrict__ slab,
                                                             int M, int S)
{
    using W = WgNat<C>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int split = (k / W::TILES) * 8 + xcd;
    int t = k % W::TILES;
    const int tap = t / (W::NT * W::NT);
    t -= tap * W::NT * W::NT;
    wgrad_nat_tile2<C, true, 4>(dz, x, rowtab, slab, M, S, split, tap, (t / W::NT) * W::BT, (t % W::NT) * W::BT,
                                smem);
}

template <int C>
__global__ __launch_bounds__(256) void wgrad_reduce_mfma_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                                int S)
{
    wgrad_reduce_mfma<C, 4>(slab, dw, S, blockIdx.x * 256 + threadIdx.x);
}

// rowtab[m] = padded row of pixel m (pv_halo.h pad_row), m < n
__global__ void rowtab_kernel(int* __restrict__ rowtab, int n)
{
    for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < n; m += gridDim.x * blockDim.x)
        rowtab[m] = (m / PIX) * PADPIX + ((m % PIX) / BOARD + 1) * PADW + (m % BOARD) + 1;
}

hipError_t launch_rowtab(int* rowtab, int n, hipStream_t st)
{
    hipLaunchKernelGGL(rowtab_kernel, dim3(256), dim3(256), 0, st, rowtab, n);
    return hipGetLastError();
}

hipError_t launch_wgrad_reduce(int C, const float* slab, float* dw, int S, hipStream_t st)
{
    const int total4 = 9 * C * C / 4;
    if (g_wgrad_variant == 1) {
        switch (C) {
            case 64: hipLaunchKernelGGL(wgrad_reduce_mfma_kernel<64>, dim3((total4 + 255) / 256), dim3(256), 0, st, slab, dw, S); break;
            case 128: hipLaunchKernelGGL(wgrad_reduce_mfma_kernel<128>, dim3((total4 + 255) / 256), dim3(256), 0, st, slab, dw, S); break;
            case 256: hipLaunchKernelGGL(wgrad_reduce_mfma_kernel<256>, dim3((total4 + 255) / 256), dim3(256), 0, st, slab, dw, S); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total4 + 255) / 256), dim3(256), 0, st, slab, dw, C, S);
    return hipGetLastError();
}

template <int C>
static hipError_t launch_wgrad_t(const float* dz, const float* x, const int* rowtab, float* slab, float* dw, int M,
                                 int S, hipStream_t st, bool reduce)
{
    using W = WgNat<C>;
    if (S % 8) return hipErrorInvalidValue;           // wgrad_splits guarantees S % 8 == 0
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           W::LDS_BYTES);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)conv3x3_wgrad_nat2<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    W::LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (g_wgrad_variant == 1) {
        if (!rowtab) return hipErrorInvalidValue;
        hipLaunchKernelGGL((conv3x3_wgrad_nat2<C>), dim3(S * W::TILES), dim3(256), W::LDS_BYTES, st, dz, x, rowtab,
                           slab, M, S);
    } else {
        hipLaunchKernelGGL((conv3x3_wgrad_nat<C>), dim3(S * W::TILES), dim3(256), W::LDS_BYTES, st, dz, x, slab, M, S);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !reduce) return e;
    return launch_wgrad_reduce(C, slab, dw, S, st);
}

// Pixel splits: S is a multiple of 8 (the XCD-aware order keeps each split on one
// XCD); the smallest S whose S * tiles workgroups fill the resident slots in ONE
// round (fewest chunks per workgroup), falling back to whole rounds for tiny M;
// every split keeps >= 2 whole 32-pixel chunks.
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
    const int slots = 256 * 2;   // two workgroups per CU
    int S = (slots / tiles) / 8 * 8;
    if (S < 8) S = 8;
    const int nch = (M + 31) / 32;
    while (S > 8 && nch < 2 * S) S -= 8;
    return S;
}

// slab must hold S*9*C*C floats, S = wgrad_splits(C, M)
hipError_t launch_wgrad(int C, const float* dz, const float* x, const int* rowtab, float* slab, float* dw, int M,
                        int S, hipStream_t st, bool reduce)
{
    switch (C) {
        case 64: return launch_wgrad_t<64>(dz, x, rowtab, slab, dw, M, S, st, reduce);
        case 128: return launch_wgrad_t<128>(dz, x, rowtab, slab, dw, M, S, st, reduce);
        case 256: return launch_wgrad_t<256>(dz, x, rowtab, slab, dw, M, S, st, reduce);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace azg
