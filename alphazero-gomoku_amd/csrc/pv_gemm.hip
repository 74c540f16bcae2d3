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
constexpr int GU = 32;                        // loads in flight per thread while staging
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
        // stage A tile [32][ldk] and B^T tile [32][ldk], zero outside the problem.
        // Batches of GU independent loads per thread are issued before their LDS
        // stores (the loads would otherwise serialise on L2 latency).
        const int tot = 32 * ldk;
        const float inv_ldk = 1.f / (float)ldk;
        auto split = [&](int e, int& r, int& k) {   // e = r*ldk + k, exact for e < 2^20
            r = (int)((float)e * inv_ldk);
            k = e - r * ldk;
            if (k < 0) { --r; k += ldk; }
            else if (k >= ldk) { ++r; k -= ldk; }
        };
        for (int e0 = 0; e0 < tot; e0 += 256 * GU) {
            float va[GU], vb[GU];
#pragma unroll
            for (int u = 0; u < GU; ++u) {
                const int e = e0 + u * 256 + tid;
                int r, k;
                if (P.sak == 1) split(e, r, k); else { k = e >> 5; r = e & 31; }
                const int i = i0 + r;
                va[u] = (e < tot && k < kc && i < P.M) ? P.A[(size_t)i * P.sai + (size_t)(k0 + k) * P.sak] : 0.f;
                int c, kb;
                if (P.sbk == 1) split(e, c, kb); else { kb = e >> 5; c = e & 31; }
                const int j = j0 + c;
                vb[u] = (e < tot && kb < kc && j < P.N) ? P.B[(size_t)(k0 + kb) * P.sbk + (size_t)j * P.sbj] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < GU; ++u) {
                const int e = e0 + u * 256 + tid;
                if (e < tot) {
                    int r, k;
                    if (P.sak == 1) split(e, r, k); else { k = e >> 5; r = e & 31; }
                    As[r * ldk + k] = va[u];
                    int c, kb;
                    if (P.sbk == 1) split(e, c, kb); else { kb = e >> 5; c = e & 31; }
                    Bs[c * ldk + kb] = vb[u];
                }
            }
        }
        __syncthreads();
        const int steps = (kc + 1) >> 1;
        const int s0 = wid * steps / 4, s1 = (wid + 1) * steps / 4;
        const float* ar = As + r32 * ldk + h;
        const float* br = Bs + r32 * ldk + h;
        for (int s = s0; s < s1; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * s], br[2 * s], acc, 0, 0, 0);
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
