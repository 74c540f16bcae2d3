// Argument blocks and launchers of the fused train-step head chain
// (pv_train_heads.hip), shared with the train-step orchestration (pv_train.hip).
#pragma once
#include "pv_internal.h"

namespace azg {

struct HeadStatsArgs {
    const float* z;        // APPLY: last block's raw bn2 input z2; else the tower output
    const float* res;      // APPLY: residual (block input)
    const float* scale;    // APPLY: bn2 scale / shift (batch statistics, finalized)
    const float* shift;
    float* aout;           // APPLY: tower output a = relu(z*s + t + res) (padded NHWC)
    const float* wpc;      // policy_conv.weight [2][C]
    const float* wvc;      // value_conv.weight [C]
    float* zh;             // [B][3][225]
    double* part;          // [nwg][6]
    int M;
    // finalize (reference BatchNorm2d train-mode forward of policy_bn / value_bn)
    const BnDesc* desc;
    int pol_layer, val_layer;
    const float* params;
    float* stats;          // running stats
    float *bmean, *binv, *bscale, *bshift;
    int64_t* nbt;
    int nbn;
};

struct HeadDgradArgs {
    const float* dlogits;  // [B][225]
    const float* dhv;      // [B][64]
    const float* wpf;      // policy_fc.weight [225][450]
    const float* wv1;      // value_fc1.weight [64][225]
    const float* fp;       // features [B][450] / [B][225] (ReLU masks)
    const float* fv;
    const float* zh;       // [B][3][225]
    const float* hmean;    // head BN mean (3)
    float *dfp, *dfv;      // masked fc data gradients
    double* part;          // [groups][6] head-BN backward sums per workgroup
    int B;
    // finalize (head_bwd_fin_wave, run by every heads_bwd_fused_kernel workgroup)
    const BnDesc* desc;
    int pol_layer, val_layer;
    const float* params;
    float* grads;
    const float* hinv;     // head BN invstd (3)
    float* hb;             // large batches: the [3][3] coefficients, written by head_bn_bwd_fin_kernel
};

struct HeadBwdArgs {
    const float* act;      // tower output a (padded NHWC)
    const float* zh;       // [B][3][225]
    const float* dfp;      // [B][450]
    const float* dfv;      // [B][225]
    const float* hmean;    // head BN mean (3)
    const float* wpc;      // policy_conv.weight [2][C]
    const float* wvc;      // value_conv.weight [C]
    float* gx;             // gradient of the tower output (padded NHWC)
    float* hpart;          // [tile][3][C] head 1x1 weight-grad partials
    // last block's bn2 backward partials (NB > 0): dy = gx * (act > 0)
    const float* z2;       // raw bn2 input
    const float* mean2;    // bn2 batch mean
    float* pa;             // [tile][C]: S dy
    float* pb;             // [tile][C]: S (z - mean) dy
    int M;
    // the head-BN backward finalize, run by every workgroup from head_dgrad_kernel's
    // dg_nwg partials; dg_nwg = 0 (batches above kHeadFoldMaxB, where every workgroup
    // re-reducing all partials would grow as B^2): read dg.hb, written by one wave before
    HeadDgradArgs dg;
    int dg_nwg;
};
constexpr int kHeadFoldMaxB = 512;

int head_dgrad_groups(int B);
int head_proj_stats_groups(int M);
hipError_t launch_head_proj_partials(int C, bool apply, const HeadStatsArgs& a, hipStream_t st);
hipError_t launch_head_bn_apply_feat(float* fp, float* fv, float* feat, int B, const HeadStatsArgs& fin,
                                     hipStream_t st);
hipError_t launch_head_dgrad(const HeadDgradArgs& a, hipStream_t st);
// one wave: the head-BN backward finalize into a.hb (B > kHeadFoldMaxB)
hipError_t launch_head_bwd_fin(const HeadDgradArgs& a, hipStream_t st);
hipError_t launch_head_fc_wgrad(const float* dlogits, const float* fp, const float* dhv, const float* fv, float* gpf,
                                float* gv1, int B, hipStream_t st);
hipError_t launch_heads_bwd_fused(int C, bool bnx, const HeadBwdArgs& a, hipStream_t st);

}  // namespace azg
