// Small strided fp32-MFMA GEMMs for the head fully-connected layers
// (network.py:104-106, 112-115) and their gradients.
//
//   C(i, j) [masked by mask(i, j) > 0] = sum_k A(i, k) * B(k, j)
//   A(i, k) = A[i*sai + k*sak],  B(k, j) = B[k*sbk + j*sbj],  C(i, j) = C[i*sci + j*scj]
//
// Every head GEMM is tiny (M <= a few thousand, N <= 450, K <= 450 or the batch),
// so one launch carries up to two problems side by side (grid.y = column tiles of
// problem 0 then problem 1).  A workgroup owns one 32x32 output tile: K is staged
// through LDS in chunks of <= 512 (row stride LDK with LDK/2 odd: conflict-free
// column reads and transposed writes), the 4 waves take contiguous quarters of a
// chunk's v_mfma_f32_32x32x2_f32 steps and the 4 partial tiles are summed in fixed
// wave order.  Deterministic, and each output row depends only on its own A row
// (batch independent when rows are boards).
#include "pv_internal.h"

namespace azg {

constexpr int GK = 512;                       // K chunk (one chunk for every head GEMM up to B = 512)
constexpr int GLDK_MAX = GK + 2;
constexpr int G_LDS = 2 * 32 * GLDK_MAX * 4;  // 131,584 B

__device__ __forceinline__ int gemm_ldk(int kc)
{
    int l = kc + (kc & 1);
    if (((l >> 1) & 1) == 0) l += 2;          // l/2 odd
    return l;
}

__global__ __launch_bounds__(256) void small_gemm_kernel(GemmPair gp)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int pi = (int)blockIdx.y < gp.ntn0 ? 0 : 1;
    const GemmProb& P = gp.p[pi];
    const int tn = (int)blockIdx.y - (pi ? gp.ntn0 : 0);
    const int i0 = blockIdx.x * 32, j0 = tn * 32;
    if (i0 >= P.M || j0 >= P.N) return;   // uniform per workgroup
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    float* As = smem;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int k0 = 0; k0 < P.K; k0 += GK) {
        const int kc = min(GK, P.K - k0);
        const int ldk = gemm_ldk(kc);
        float* Bs = smem + 32 * ldk;
        // stage A tile [32][ldk] and B^T tile [32][ldk], zero outside the problem (the
        // pad column k = kc of an odd chunk included).  Each thread owns one tile row
        // and a k stride of 8 (k-contiguous operands: 8 threads per row read 32-B runs)
        // or one k phase and a row (row-contiguous operands: 32 threads read a 128-B
        // row of the other dimension); no per-element index division, UNR loads in
        // flight per thread before their LDS stores.
        constexpr int UNR = 16;
        struct Op { const float* src; float* d; bool rok; int sx_k; int kq; };
        auto op = [&](const float* X, int sx_row, int sx_k, int rlim, int rbase, float* dst) {
            const bool kcontig = sx_k == 1;
            const int r = kcontig ? (tid >> 3) : (tid & 31);
            const int kq = kcontig ? (tid & 7) : (tid >> 5);
            return Op{X + (size_t)(rbase + r) * sx_row + (size_t)k0 * sx_k, dst + r * ldk, rbase + r < rlim, sx_k, kq};
        };
        const Op oa = op(P.A, P.sai, P.sak, P.M, i0, As), ob = op(P.B, P.sbj, P.sbk, P.N, j0, Bs);
        const int kend = kc + (kc & 1);
        // both operands' loads of a step in flight together (UNR each), then their stores
        for (int kb = 0; kb < kend; kb += 8 * UNR) {
            float va[UNR], vb[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int ka = kb + oa.kq + 8 * u, kbb = kb + ob.kq + 8 * u;
                va[u] = (oa.rok && ka < kc) ? oa.src[(size_t)ka * oa.sx_k] : 0.f;
                vb[u] = (ob.rok && kbb < kc) ? ob.src[(size_t)kbb * ob.sx_k] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int ka = kb + oa.kq + 8 * u, kbb = kb + ob.kq + 8 * u;
                if (ka < kend) oa.d[ka] = va[u];
                if (kbb < kend) ob.d[kbb] = vb[u];
            }
        }
        __syncthreads();
        const int steps = (kc + 1) >> 1;
        const int s0 = wid * steps / 4, s1 = (wid + 1) * steps / 4;
        const float* ar = As + r32 * ldk + h;
        const float* br = Bs + r32 * ldk + h;
        int s = s0;
        for (; s + 4 <= s1; s += 4) {   // 4 steps' fragments read ahead of their MFMAs
            float a4[4], b4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a4[u] = ar[2 * (s + u)];
                b4[u] = br[2 * (s + u)];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[u], b4[u], acc, 0, 0, 0);
        }
        for (; s < s1; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * s], br[2 * s], acc, 0, 0, 0);
        __syncthreads();
    }
    float* red = smem;   // [4][16][64]
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(wid * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    if (wid == 0) {
        const int j = j0 + r32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = red[r * 64 + lane];
            v += red[(16 + r) * 64 + lane];
            v += red[(32 + r) * 64 + lane];
            v += red[(48 + r) * 64 + lane];
            const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (i < P.M && j < P.N) {
                if (P.mask && !(P.mask[(size_t)i * P.smi + (size_t)j * P.smj] > 0.f)) v = 0.f;
                P.C[(size_t)i * P.sci + (size_t)j * P.scj] = v;
            }
        }
    }
}

hipError_t launch_small_gemm(const GemmProb& p0, const GemmProb* p1, hipStream_t st)
{
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute((const void*)small_gemm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           G_LDS);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    GemmPair gp;
    gp.p[0] = p0;
    gp.p[1] = p1 ? *p1 : p0;
    gp.ntn0 = (p0.N + 31) / 32;
    const int ntn1 = p1 ? (p1->N + 31) / 32 : 0;
    const int mt = (max(p0.M, p1 ? p1->M : 0) + 31) / 32;
    if (mt == 0 || gp.ntn0 + ntn1 == 0) return hipSuccess;
    hipLaunchKernelGGL(small_gemm_kernel, dim3(mt, gp.ntn0 + ntn1), dim3(256), G_LDS, st, gp);
    return hipGetLastError();
}

}  // namespace azg
