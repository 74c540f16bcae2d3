// Weight re-packing and BatchNorm folding (run when parameters change).
//
// Torch layouts in (network.py:41-73): conv [Cout][Cin][3][3], linear [out][in].
// Packed layouts out:
//   res conv  -> wp[kc][n][32], kc = tap*(C/32) + cin/32, tap = ky*3 + kx
//   dgrad     -> wd[kc][n=cin][32 of cout] for the flipped tap 8 - tap (transpose
//                conv: dX[ci] at q = sum over taps and cout of dY[co] at q + off(t') W[co][ci][2-ky'][2-kx'])
//   stem      -> ws[k][c], k = cin*9 + ky*3 + kx
//   FC        -> W^T [in][out]
// Eval-mode BN fold, as ATen's CPU inference path (alpha = invstd*gamma,
// beta = bias - mean*alpha, y = x*alpha + beta):
//   invstd = 1/sqrt(running_var + eps)
#include "pv_internal.h"

namespace azg {


// All residual convs at once: layer l = blockIdx.y reads params + offs[l] and
// writes the forward packing to wp + l*9*C*C and, when wd is given, the dgrad
// packing to wd + l*9*C*C (one launch instead of 2 per layer).
__global__ void pack_convs_kernel(const float* __restrict__ params, const int64_t* __restrict__ offs,
                                  float* __restrict__ wp, float* __restrict__ wd, int C)
{
    const int total = 9 * C * C;
    const int cg_n = C / 32;
    const float* w = params + offs[blockIdx.y];
    float* wpl = wp + (size_t)blockIdx.y * total;
    float* wdl = wd ? wd + (size_t)blockIdx.y * total : nullptr;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const int k = idx & 31;
        const int n = (idx >> 5) % C;
        const int kc = idx / (32 * C);
        const int tap = kc / cg_n, cg = kc - tap * cg_n;
        const int c2 = cg * 32 + k;
        wpl[idx] = w[(n * C + c2) * 9 + tap];                 // = pack_conv3x3_kernel
        if (wdl) wdl[idx] = w[(c2 * C + n) * 9 + (8 - tap)];  // = pack_dgrad_kernel
    }
}

__global__ void pack_stem_kernel(const float* __restrict__ w, float* __restrict__ ws, int C)
{
    const int total = 27 * C;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const int c = idx % C, k = idx / C;
        ws[idx] = w[c * 27 + k];
    }
}

__global__ void transpose_kernel(const float* __restrict__ src, float* __restrict__ dst, int R, int Cc)
{
    const int total = R * Cc;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const int r = idx / Cc, c = idx - r * Cc;
        dst[c * R + r] = src[idx];
    }
}

__global__ void fold_bn_kernel(const float* __restrict__ params, const float* __restrict__ stats,
                               const BnDesc* __restrict__ desc, float* __restrict__ scale,
                               float* __restrict__ shift)
{
    const BnDesc d = desc[blockIdx.x];
    for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
        const float invstd = 1.0f / sqrtf(stats[d.stat_off + d.c + c] + BN_EPS);
        const float alpha = invstd * params[d.gamma_off + c];
        scale[d.out_off + c] = alpha;
        shift[d.out_off + c] = params[d.beta_off + c] - stats[d.stat_off + c] * alpha;
    }
}

// Every re-pack of repack() in ONE launch (it runs at the start of every train step,
// on the critical path): blockIdx.y < nl packs residual conv l (as pack_convs_kernel),
// y == nl the stem, y == nl + 1 the head FCs, y == nl + 2 folds the eval BN (one
// layer per blockIdx.x).  Same per-element arithmetic as the separate kernels.
struct RepackArgs {
    const float* params;
    const int64_t* conv_offs;
    float* wp;
    float* wd;
    int C, nl;
    const float* stem_w;
    float* ws;
    const float* wpf;
    const float* wv1;
    float* wfc;
    const float* stats;
    const BnDesc* desc;
    int nbn;
    float* scale;
    float* shift;
    int y0;       // first section of this launch (grid.y covers y0 .. y0 + grid.y - 1)
    int skip;     // a section to skip (-1: none)
};

__global__ __launch_bounds__(256) void repack_all_kernel(const RepackArgs a)
{
    const int y = a.y0 + (int)blockIdx.y;
    if (y == a.skip) return;
    const int C = a.C;
    const int stride = gridDim.x * blockDim.x;
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (y < a.nl) {
        const int total = 9 * C * C, cg_n = C / 32;
        const float* w = a.params + a.conv_offs[y];
        float* wpl = a.wp + (size_t)y * total;
        float* wdl = a.wd ? a.wd + (size_t)y * total : nullptr;
        for (int idx = i0; idx < total; idx += stride) {
            const int k = idx & 31, n = (idx >> 5) % C, kc = idx / (32 * C);
            const int tap = kc / cg_n, c2 = (kc - tap * cg_n) * 32 + k;
            wpl[idx] = w[(n * C + c2) * 9 + tap];
            if (wdl) wdl[idx] = w[(c2 * C + n) * 9 + (8 - tap)];
        }
    } else if (y == a.nl) {
        for (int idx = i0; idx < 27 * C; idx += stride) a.ws[idx] = a.stem_w[(idx % C) * 27 + idx / C];
    } else if (y == a.nl + 1) {
        for (int idx = i0; idx < FC_OUT * FC_KP; idx += stride) {
            const int j = idx / FC_KP, k = idx - j * FC_KP;
            float v = 0.f;
            if (j < ACTIONS) {
                if (k < 2 * PIX) v = a.wpf[j * 2 * PIX + k];
            } else if (k < PIX) {
                v = a.wv1[(j - ACTIONS) * PIX + k];
            }
            a.wfc[idx] = v;
        }
    } else if (blockIdx.x < (unsigned)a.nbn) {
        const BnDesc d = a.desc[blockIdx.x];
        for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
            const float invstd = 1.0f / sqrtf(a.stats[d.stat_off + d.c + c] + BN_EPS);
            const float alpha = invstd * a.params[d.gamma_off + c];
            a.scale[d.out_off + c] = alpha;
            a.shift[d.out_off + c] = a.params[d.beta_off + c] - a.stats[d.stat_off + c] * alpha;
        }
    }
}

// part: 0 every section; 1 the stem only (y = nl); 2 the residual convs (+ dgrad packs)
// and the head FCs -- neither the stem nor the eval BN fold (the train step's split
// repack: part 1 on the caller's stream, part 2 on the side stream)
hipError_t launch_repack_all(const float* params, const int64_t* conv_offs, int nl, float* wp, float* wd, int C,
                             const float* stem_w, float* ws, const float* wpf, const float* wv1, float* wfc,
                             const float* stats, const void* desc, int nbn, float* scale, float* shift,
                             hipStream_t st, int part)
{
    RepackArgs a{params, conv_offs, wp, wd, C, nl, stem_w, ws, wpf, wv1, wfc, stats, (const BnDesc*)desc, nbn,
                 scale, shift, part == 1 ? nl : 0, part == 2 ? nl : -1};
    int nb = (9 * C * C + 255) / 256;
    nb = nb > 256 ? 256 : nb;
    nb = nb < nbn ? nbn : nb;
    if (part == 1) nb = (27 * C + 255) / 256;
    hipLaunchKernelGGL(repack_all_kernel, dim3(nb, part == 1 ? 1 : part == 2 ? nl + 2 : nl + 3), dim3(256), 0, st, a);
    return hipGetLastError();
}

static inline int nblk(int total) { int b = (total + 255) / 256; return b > 4096 ? 4096 : b; }

// ---- split-fp16 (H3) eval weights (pv_halo.h halo_tile VAR bit 64) ----
// e_l = 14 - floor(log2 max|w_l|): max|w_l| * 2^e < 2^15, so hi = fp16(w 2^e) never
// overflows and the lo parts of every weight above 2^-10 of the layer's largest stay
// normal fp16 (the rest carry 2^-25 absolute error).  The max runs on H3_MAXB workgroups
// per layer (float4 loads, one atomicMax on the bits of a non-negative float: their
// order is the floats' order); exps[l] holds those bits until scale_h3_kernel turns them
// into e_l (the train step re-packs every step: one workgroup per layer took 90 us).
constexpr int H3_MAXB = 32;
__device__ __forceinline__ int h3_exp_of(unsigned maxbits)
{
    const float m = __uint_as_float(maxbits);
    return m > 0.f ? 14 - ilogbf(m) : 0;
}
__global__ __launch_bounds__(256) void h3_max_kernel(const float* __restrict__ params, const int64_t* __restrict__ offs,
                                                     int C, unsigned* __restrict__ maxbits)
{
    __shared__ float red[256];
    const int l = blockIdx.y;
    const float* wl = params + offs[l];
    float m = 0.f;
    if ((offs[l] & 3) == 0) {   // the conv weights of the parameter layout start 16-B aligned (C % 32 == 0)
        const f32x4* w = (const f32x4*)wl;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < 9 * C * C / 4; i += H3_MAXB * 256) {
            const f32x4 v = w[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
    } else {
        for (int i = blockIdx.x * 256 + threadIdx.x; i < 9 * C * C; i += H3_MAXB * 256) m = fmaxf(m, fabsf(wl[i]));
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(maxbits + l, __float_as_uint(red[0]));
}

// packed row (kc * C + n) of 32 K values -> 64 halves [hi 32 | lo 32] of w * 2^e, in
// the fp32 packing's order (repack_all_kernel)
__global__ __launch_bounds__(256) void pack_h3_kernel(const float* __restrict__ params, const int64_t* __restrict__ offs,
                                                      int C, const unsigned* __restrict__ maxbits,
                                                      _Float16* __restrict__ out)
{
    const int total = 9 * C * C, cg_n = C / 32;
    const int l = blockIdx.y;
    const float* w = params + offs[l];
    _Float16* o = out + (size_t)l * 2 * total;
    const float sc = ldexpf(1.f, h3_exp_of(maxbits[l]));
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
        const int k = idx & 31, n = (idx >> 5) % C, kc = idx / (32 * C);
        const int tap = kc / cg_n, c2 = (kc - tap * cg_n) * 32 + k;
        const float v = w[(n * C + c2) * 9 + tap] * sc;
        const _Float16 hi = (_Float16)v;
        const int row = idx >> 5;
        o[row * 64 + k] = hi;
        o[row * 64 + 32 + k] = (_Float16)(v - (float)hi);
    }
}

// scale16 = the eval BN scale of every residual conv's BN times 2^-e (exact); inv (train
// forward, optional) = 2^-e per layer and output channel: the raw conv output's factor;
// exps[l] <- e_l (it held the max bits)
__global__ void scale_h3_kernel(const float* __restrict__ scale, const int* __restrict__ conv_bn_off,
                                int* __restrict__ exps, int C, float* __restrict__ scale16,
                                float* __restrict__ inv)
{
    const int l = blockIdx.x, o = conv_bn_off[l];
    const int e = h3_exp_of((unsigned)exps[l]);
    __syncthreads();   // every thread has read the bits before thread 0 replaces them
    const float f = ldexpf(1.f, -e);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        scale16[o + c] = scale[o + c] * f;
        if (inv) inv[l * C + c] = f;
    }
    if (threadIdx.x == 0) exps[l] = e;
}

hipError_t launch_pack_h3(const float* params, const int64_t* offs, int nl, int C, const int* conv_bn_off,
                          const float* scale, int* exps, void* wp16, float* scale16, float* inv, hipStream_t st)
{
    if (nl <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(exps, 0, (size_t)nl * sizeof(int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(h3_max_kernel, dim3(H3_MAXB, nl), dim3(256), 0, st, params, offs, C, (unsigned*)exps);
    int nb = nblk(9 * C * C);
    nb = nb > 256 ? 256 : nb;
    hipLaunchKernelGGL(pack_h3_kernel, dim3(nb, nl), dim3(256), 0, st, params, offs, C, (const unsigned*)exps,
                       (_Float16*)wp16);
    hipLaunchKernelGGL(scale_h3_kernel, dim3(nl), dim3(256), 0, st, scale, conv_bn_off, exps, C, scale16, inv);
    return hipGetLastError();
}

// the split-fp16 dgrad packing (key 50): pack_h3's rows for the flipped, transposed taps
// of pack_convs_kernel's wd (row kc * C + n = cin n, K values = 32 couts of group kc % CG
// at tap 8 - kc / CG), w * 2^e with the layer's e (exps, after scale_h3_kernel)
__global__ __launch_bounds__(256) void pack_h3_dgrad_kernel(const float* __restrict__ params,
                                                            const int64_t* __restrict__ offs, int C,
                                                            const int* __restrict__ exps, _Float16* __restrict__ out)
{
    const int total = 9 * C * C, cg_n = C / 32;
    const int l = blockIdx.y;
    const float* w = params + offs[l];
    _Float16* o = out + (size_t)l * 2 * total;
    const float sc = ldexpf(1.f, exps[l]);
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
        const int k = idx & 31, n = (idx >> 5) % C, kc = idx / (32 * C);
        const int tap = kc / cg_n, c2 = (kc - tap * cg_n) * 32 + k;
        const float v = w[(c2 * C + n) * 9 + (8 - tap)] * sc;
        const _Float16 hi = (_Float16)v;
        const int row = idx >> 5;
        o[row * 64 + k] = hi;
        o[row * 64 + 32 + k] = (_Float16)(v - (float)hi);
    }
}

hipError_t launch_pack_h3_dgrad(const float* params, const int64_t* offs, int nl, int C, const int* exps, void* wd16,
                                hipStream_t st)
{
    if (nl <= 0) return hipSuccess;
    int nb = nblk(9 * C * C);
    nb = nb > 256 ? 256 : nb;
    hipLaunchKernelGGL(pack_h3_dgrad_kernel, dim3(nb, nl), dim3(256), 0, st, params, offs, C, exps, (_Float16*)wd16);
    return hipGetLastError();
}

hipError_t launch_pack_convs(const float* params, const int64_t* offs, int nl, float* wp, float* wd, int C,
                             hipStream_t st)
{
    int nb = nblk(9 * C * C);
    nb = nb > 256 ? 256 : nb;
    hipLaunchKernelGGL(pack_convs_kernel, dim3(nb, nl), dim3(256), 0, st, params, offs, wp, wd, C);
    return hipGetLastError();
}

hipError_t launch_pack_stem(const float* w, float* ws, int C, hipStream_t st)
{
    hipLaunchKernelGGL(pack_stem_kernel, dim3(nblk(27 * C)), dim3(256), 0, st, w, ws, C);
    return hipGetLastError();
}

// head FC weights -> wfc[FC_OUT][FC_KP] (pv_common.h): policy_fc rows (K = 450) then
// value_fc1 rows (K = 225), zero-padded to FC_KP
__global__ void pack_fc_kernel(const float* __restrict__ wpf, const float* __restrict__ wv1, float* __restrict__ wfc)
{
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < FC_OUT * FC_KP; idx += gridDim.x * blockDim.x) {
        const int j = idx / FC_KP, k = idx - j * FC_KP;
        float v = 0.f;
        if (j < ACTIONS) {
            if (k < 2 * PIX) v = wpf[j * 2 * PIX + k];
        } else if (k < PIX) {
            v = wv1[(j - ACTIONS) * PIX + k];
        }
        wfc[idx] = v;
    }
}

hipError_t launch_pack_fc(const float* wpf, const float* wv1, float* wfc, hipStream_t st)
{
    hipLaunchKernelGGL(pack_fc_kernel, dim3(nblk(FC_OUT * FC_KP)), dim3(256), 0, st, wpf, wv1, wfc);
    return hipGetLastError();
}

hipError_t launch_transpose(const float* src, float* dst, int R, int Cc, hipStream_t st)
{
    hipLaunchKernelGGL(transpose_kernel, dim3(nblk(R * Cc)), dim3(256), 0, st, src, dst, R, Cc);
    return hipGetLastError();
}

hipError_t launch_fold_bn(const float* params, const float* stats, const void* desc, int nlayers,
                          float* scale, float* shift, hipStream_t st)
{
    hipLaunchKernelGGL(fold_bn_kernel, dim3(nlayers), dim3(256), 0, st, params, stats,
                       (const BnDesc*)desc, scale, shift);
    return hipGetLastError();
}

}  // namespace azg
