// Split-fp16 (H3) residual-conv tile lab (round 5).
//
// Stand-alone executable: times per-layer launches of halo_tile (pv_halo.h, VAR bit 64)
// at several tile shapes / register blockings on synthetic operands (padded NHWC
// activations with a zero halo, split fp16 weights in the pack_h3 layout), reports
// device time per launch (hipEvents), fp32-equivalent TFLOP/s, and whether every
// variant's output is bitwise the first variant's (all shapes share the per-element K
// order).  Not linked into the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I alphazero-gomoku_amd/csrc \
//       scripts/h3_lab.hip -o scripts/h3_lab
//   scripts/h3_lab <C> <boards> <reps>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <string>

#include "pv_halo.h"
#include "pv_h3.h"

using namespace azg;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <int C, int BN_, int WM_, int TM_, int NW_, int VAR, int WPE>
__global__ __launch_bounds__(64 * NW_, WPE) void lab_conv(const float* __restrict__ in, const float* __restrict__ wp,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ resid, float* __restrict__ out,
                                                          int M, H3Guard guard)
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NTN = C / T::BN;
    const int L = blockIdx.x, nt = gridDim.x;
    const int xcd = L & 7, q8 = nt >> 3, r8 = nt & 7;
    const int t = xcd * q8 + min(xcd, r8) + (L >> 3);
    halo_tile<C, BN_, WM_, TM_, NW_, EPI_BN_RES_RELU, false, 0, VAR>(
        in, wp, scale, shift, resid, out, __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000), M,
        (t / NTN) * T::BM, (t % NTN) * T::BN, smem, EpiX{}, ProX{}, FinX{}, guard);
}

template <int C, int BN_, int WM_, int TM_, int NW_, int TPS, int NWB, int WPE, int ABL = 0>
__global__ __launch_bounds__(64 * NW_, WPE) void lab_h3(const float* __restrict__ in, const float* __restrict__ wp,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ resid, float* __restrict__ out,
                                                        int M, H3Guard guard)
{
    using T = ConvTile<C, BN_, WM_, TM_, NW_>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NTN = C / T::BN;
    const int L = blockIdx.x, nt = gridDim.x;
    const int xcd = L & 7, q8 = nt >> 3, r8 = nt & 7;
    const int t = xcd * q8 + min(xcd, r8) + (L >> 3);
    h3_tile<C, BN_, WM_, TM_, NW_, TPS, NWB, EPI_BN_RES_RELU, false, 0, ABL & 7, ABL & ~7>(
        in, wp, scale, shift, resid, out, __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000), M,
        (t / NTN) * T::BM, (t % NTN) * T::BN, smem, guard);
}

struct Variant {
    std::string name;
    int C;
    int bm, bn;
    size_t lds;
    void (*launch)(const float*, const float*, const float*, const float*, const float*, float*, int, H3Guard,
                   hipStream_t);
    hipError_t (*prep)();
};

template <int C, int BN, int WM, int TM, int NW, int VAR, int WPE>
static void launch_v(const float* in, const float* wp, const float* sc, const float* sh, const float* rs, float* out,
                     int M, H3Guard g, hipStream_t st)
{
    using T = ConvTile<C, BN, WM, TM, NW>;
    constexpr int lds = halo_lds_bytes<C, BN, WM, TM, NW, VAR>();
    dim3 grid(((M + T::BM - 1) / T::BM) * (C / T::BN));
    hipLaunchKernelGGL((lab_conv<C, BN, WM, TM, NW, VAR, WPE>), grid, dim3(T::NT), lds, st, in, wp, sc, sh, rs, out,
                       M, g);
}
template <int C, int BN, int WM, int TM, int NW, int VAR, int WPE>
static hipError_t prep_v()
{
    constexpr int lds = halo_lds_bytes<C, BN, WM, TM, NW, VAR>();
    return hipFuncSetAttribute((const void*)lab_conv<C, BN, WM, TM, NW, VAR, WPE>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int WPE, int ABL = 0>
static void launch_h(const float* in, const float* wp, const float* sc, const float* sh, const float* rs, float* out,
                     int M, H3Guard g, hipStream_t st)
{
    using T = ConvTile<C, BN, WM, TM, NW>;
    constexpr int lds = h3_lds_bytes<C, BN, WM, TM, NW, TPS, NWB, ABL & ~7>();
    dim3 grid(((M + T::BM - 1) / T::BM) * (C / T::BN));
    hipLaunchKernelGGL((lab_h3<C, BN, WM, TM, NW, TPS, NWB, WPE, ABL>), grid, dim3(T::NT), lds, st, in, wp, sc, sh, rs,
                       out, M, g);
}
template <int C, int BN, int WM, int TM, int NW, int TPS, int NWB, int WPE, int ABL = 0>
static hipError_t prep_h()
{
    constexpr int lds = h3_lds_bytes<C, BN, WM, TM, NW, TPS, NWB, ABL & ~7>();
    return hipFuncSetAttribute((const void*)lab_h3<C, BN, WM, TM, NW, TPS, NWB, WPE, ABL>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}
#define VH(C, BN, WM, TM, NW, TPS, NWB, WPE)                                                                        \
    Variant{"h3_tile " #BN "x" #WM "x" #TM " nw" #NW " tps" #TPS " nwb" #NWB " wpe" #WPE, C,                      \
            ConvTile<C, BN, WM, TM, NW>::BM, BN, (size_t)H3Tile<C, BN, WM, TM, NW, TPS, NWB>::LDS,                  \
            launch_h<C, BN, WM, TM, NW, TPS, NWB, WPE>, prep_h<C, BN, WM, TM, NW, TPS, NWB, WPE>}
#define VA(C, BN, WM, TM, NW, TPS, NWB, WPE, ABL)                                                                   \
    Variant{"h3_tile " #BN "x" #WM "x" #TM " nw" #NW " tps" #TPS " nwb" #NWB " wpe" #WPE " ABLATION " #ABL, C,     \
            ConvTile<C, BN, WM, TM, NW>::BM, BN, (size_t)h3_lds_bytes<C, BN, WM, TM, NW, TPS, NWB, ABL & ~7>(),            \
            launch_h<C, BN, WM, TM, NW, TPS, NWB, WPE, ABL>, prep_h<C, BN, WM, TM, NW, TPS, NWB, WPE, ABL>}
#define V(C, BN, WM, TM, NW, VAR, WPE)                                                                              \
    Variant{#BN "x" #WM "x" #TM " nw" #NW " var" #VAR " wpe" #WPE, C, ConvTile<C, BN, WM, TM, NW>::BM, BN,         \
            (size_t)halo_lds_bytes<C, BN, WM, TM, NW, VAR>(), launch_v<C, BN, WM, TM, NW, VAR, WPE>,                \
            prep_v<C, BN, WM, TM, NW, VAR, WPE>}

template <int C>
static std::vector<Variant> variants()
{
    return {
        V(C, 64, 4, 1, 8, 99, 2),    // product per-layer form: 128x64, 8 waves, wave 32x32
        V(C, 128, 2, 2, 4, 99, 2),   // 128x128, 4 waves as 2x2, wave 64x64
        // h3_tile (pv_h3.h): LDS-DMA weight stages, counted waits, raw barriers
        VH(C, 64, 4, 1, 8, 1, 2, 4),     // 128x64, wave 32x32, 1-tap stages
        VH(C, 64, 4, 1, 8, 1, 3, 4),     // ... three stage buffers
        VH(C, 64, 4, 1, 8, 3, 2, 2),     // ... 3-tap stages (one workgroup per CU by LDS)
        VH(C, 128, 2, 2, 4, 1, 2, 2),    // 128x128, wave 64x64, 1-tap stages
        VH(C, 128, 2, 2, 4, 1, 3, 2),    // ... three stage buffers
        VH(C, 128, 4, 1, 8, 1, 2, 2),    // 128x128, 8 waves, wave 32x64
        VH(C, 128, 2, 2, 8, 1, 2, 2),    // 128x128, 8 waves as 2x4, wave 64x32
        VH(C, 128, 2, 2, 4, 3, 2, 1),    // 128x128, wave 64x64, 3-tap stages, one workgroup per CU
        // OPT (ablation value bits >= 8): 8 = next-group halo loads at the group's first stage,
        // 16 = epilogue residual loads before the LDS pass -- bitwise identical
        VA(C, 128, 2, 2, 4, 1, 3, 2, 8), VA(C, 128, 2, 2, 4, 1, 3, 2, 16), VA(C, 128, 2, 2, 4, 1, 3, 2, 24),
        VA(C, 64, 4, 1, 8, 3, 2, 2, 8), VA(C, 64, 4, 1, 8, 3, 2, 2, 24), VA(C, 64, 4, 1, 8, 1, 3, 4, 24),
        // OPT 32: direct epilogue (no LDS pass)
        VA(C, 128, 2, 2, 4, 1, 3, 2, 32), VA(C, 128, 4, 1, 8, 1, 2, 4, 32), VA(C, 64, 4, 1, 8, 3, 2, 2, 32),
        // 128x128 / 8 waves (wave 32x64) capped at 128 VGPRs: two workgroups per CU
        VH(C, 128, 4, 1, 8, 1, 2, 4), VH(C, 128, 4, 1, 8, 1, 3, 4), VA(C, 128, 4, 1, 8, 1, 3, 4, 8),
        VH(C, 128, 2, 2, 8, 1, 3, 4),
        // timing ablations (results invalid): 1 no epilogue, 2 no halo loads, 7 neither nor weights
        VA(C, 128, 2, 2, 4, 1, 3, 2, 1), VA(C, 128, 2, 2, 4, 1, 3, 2, 2), VA(C, 128, 2, 2, 4, 1, 3, 2, 7),
    };
}

static uint32_t lcg(uint64_t& s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
}

template <int C>
static int run(int B, int reps)
{
    const int M = B * PIX;
    const size_t act = (size_t)B * PADPIX * C;
    std::vector<float> h_in(act, 0.f), h_res(act, 0.f);
    uint64_t s = 12345;
    for (int b = 0; b < B; ++b)
        for (int y = 1; y <= BOARD; ++y)
            for (int x = 1; x <= BOARD; ++x)
                for (int c = 0; c < C; ++c) {
                    const size_t o = ((size_t)b * PADPIX + y * PADW + x) * C + c;
                    h_in[o] = (lcg(s) & 0xffff) / 65536.f * ((lcg(s) & 3) ? 1.f : 0.f);   // ReLU-like
                    h_res[o] = (lcg(s) & 0xffff) / 65536.f;
                }
    // split fp16 weights: [kchunk][n][hi 32 | lo 32] halves, scaled into fp16 range
    const size_t wn = (size_t)9 * C * C;
    std::vector<_Float16> h_w(2 * wn);
    for (size_t i = 0; i < wn; ++i) {
        const float v = ((float)(lcg(s) & 0xffff) / 65536.f - 0.5f) * 4096.f;
        const _Float16 hi = (_Float16)v;
        h_w[(i >> 5) * 64 + (i & 31)] = hi;
        h_w[(i >> 5) * 64 + 32 + (i & 31)] = (_Float16)(v - (float)hi);
    }
    std::vector<float> h_sc(C), h_sh(C);
    for (int c = 0; c < C; ++c) {
        h_sc[c] = 1.f / 4096.f / (float)(9 * C) * 4.f;
        h_sh[c] = ((lcg(s) & 0xff) / 256.f - 0.5f) * 0.1f;
    }
    float *d_in, *d_res, *d_out, *d_ref, *d_sc, *d_sh;
    void* d_w;
    unsigned* d_ring;
    CK(hipMalloc(&d_in, act * 4));
    CK(hipMalloc(&d_res, act * 4));
    CK(hipMalloc(&d_out, act * 4));
    CK(hipMalloc(&d_ref, act * 4));
    CK(hipMalloc(&d_w, 2 * wn * 2));
    CK(hipMalloc(&d_sc, C * 4));
    CK(hipMalloc(&d_sh, C * 4));
    CK(hipMalloc(&d_ring, kH3RingSize * 4));
    CK(hipMemcpy(d_in, h_in.data(), act * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_res, h_res.data(), act * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w, h_w.data(), 2 * wn * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sc, h_sc.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sh, h_sh.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_ring, 0, kH3RingSize * 4));
    CK(hipMemset(d_out, 0, act * 4));
    CK(hipMemset(d_ref, 0, act * 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const H3Guard g{d_ring, 7};
    const double flop = 2.0 * M * C * 9.0 * C;
    auto vs = variants<C>();
    std::vector<float> h_out(act), h_ref(act);
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        Variant& v = vs[vi];
        if (v.lds > 160 * 1024) {
            printf("{\"C\": %d, \"B\": %d, \"variant\": \"%s\", \"skipped\": \"lds %zu\"}\n", C, B, v.name.c_str(),
                   v.lds);
            continue;
        }
        CK(v.prep());
        float* dst = vi == 0 ? d_ref : d_out;
        CK(hipMemsetAsync(dst, 0, act * 4, st));
        v.launch(d_in, (const float*)d_w, d_sc, d_sh, d_res, dst, M, g, st);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        float best = 1e30f, tot = 0.f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < reps; ++i) v.launch(d_in, (const float*)d_w, d_sc, d_sh, d_res, dst, M, g, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            best = ms < best ? ms : best;
            tot += ms;
        }
        bool same = true;
        double maxd = 0.0;
        if (vi > 0) {
            CK(hipMemcpy(h_out.data(), d_out, act * 4, hipMemcpyDeviceToHost));
            same = memcmp(h_out.data(), h_ref.data(), act * 4) == 0;
            for (size_t i = 0; i < act; ++i) {
                const double d = fabs((double)h_out[i] - (double)h_ref[i]);
                maxd = d > maxd ? d : maxd;
            }
        } else {
            CK(hipMemcpy(h_ref.data(), d_ref, act * 4, hipMemcpyDeviceToHost));
        }
        unsigned ring[kH3RingSize];
        CK(hipMemcpy(ring, d_ring, sizeof(ring), hipMemcpyDeviceToHost));
        int posted = 0;
        for (unsigned k = 0; k < kH3RingSize; ++k) posted += ring[k] != 0;
        printf("{\"C\": %d, \"B\": %d, \"variant\": \"%s\", \"tile\": \"%dx%d\", \"lds\": %zu, \"best_us\": %.2f, "
               "\"mean_us\": %.2f, \"tflops\": %.1f, \"bitwise_first\": %s, \"max_abs_diff\": %.3g, \"posted\": %d}\n",
               C, B, v.name.c_str(), v.bm, v.bn, v.lds, best * 1e3, tot / 3 * 1e3, flop / (best * 1e-3) / 1e12,
               same ? "true" : "false", maxd, posted);
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv)
{
    const int C = argc > 1 ? atoi(argv[1]) : 128;
    const int B = argc > 2 ? atoi(argv[2]) : 4096;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    if (B < 1 || B > 8192 || reps < 1 || reps > 1000) {
        fprintf(stderr, "bad args\n");
        return 2;
    }
    if (C == 128) return run<128>(B, reps);
    if (C == 256) return run<256>(B, reps);
    fprintf(stderr, "C must be 128 or 256\n");
    return 2;
}
