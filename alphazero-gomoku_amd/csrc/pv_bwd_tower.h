// Persistent train backward (pv_bwd_tower.hip): the descriptor of one backward conv
// and the launcher, shared with the train-step orchestration (pv_train.hip).
#pragma once
#include "pv_internal.h"
#include "pv_halo.h"

namespace azg {

// One conv of the tower backward, in processing order p (conv2 of the last block
// first).  Stages (reference autograd of network.py:12-25 through loss.backward(),
// network.py:224):
//   A  dz = BatchNorm backward of the conv's output BN applied to the gradient g of
//      its BN + ReLU output (bn_bwd_apply_kernel arithmetic; act == nullptr: the ReLU
//      mask comes from z * fscale + fshift, the residual-free layers);
//   D  out = conv(dz, flipped W) [+ resid], with the BatchNorm-backward partial sums of
//      the layer below in the epilogue and their finalize by the last workgroup of each
//      N tile (pv_halo.h XE_BNBWD + FinX, fx.done published in-launch);
//   W  slab = split-K partials of dW = dz^T . X(tap) (pv_wgrad.h wgrad_nat_tile);
//   R  dw (torch layout) = the slabs summed in fixed order (pv_wgrad.h).
struct BwdConv {
    const float* g;
    const float* act;
    const float* z;
    const float* mean;
    const float* gm;
    const float* kk;
    const float* iw;
    const float* fscale;
    const float* fshift;
    float* dz;
    float* gres;          // conv2 of a block: dy (the residual gradient) also written here
    const float* wd;      // dgrad-packed weights
    const float* resid;   // conv1 of a block: the residual gradient added to the dgrad
    float* out;
    EpiX ex;
    FinX fx;
    const float* wx;      // the conv's forward input (weight-grad operand)
    float* slab;
    float* dw;
};

constexpr int kBwdSyncHead = 8;   // sync words: [0] work counter, [1] error, [2] exits
// sync words of a launch over nconv convs: per conv p four counters at
// kBwdSyncHead + 4p: A items done, W items done, R items done, finalizes published
// (fin of conv p is published by conv p-1's dgrad; conv nconv's by the last one)
constexpr int bwd_sync_words(int nconv) { return kBwdSyncHead + 4 * (nconv + 1); }
inline unsigned* bwd_fin_word(unsigned* sync, int p) { return sync + kBwdSyncHead + 4 * p + 3; }

// desc: device array of nconv BwdConv; sync: bwd_sync_words(nconv) words, zero at the
// first launch (every launch leaves them zero)
// trace (timing studies, AZG_BWD_TRACE): bwd_tower_items() x 5 u64 {claim, workgroup,
// start, dependencies met, end} (wall_clock64, 100 MHz), or null
int bwd_tower_items(int C, int nconv, int M, int S);
hipError_t launch_bwd_tower(int C, const BwdConv* desc, int nconv, int M, int S, unsigned* sync, unsigned* status,
                            hipStream_t st, unsigned long long* trace = nullptr);

}  // namespace azg
