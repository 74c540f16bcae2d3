/*
 * azg_pv.h -- C-ABI of the MI355X (gfx950) policy/value engine.
 *
 * The reference has no FFI layer: its boundary is Python duck typing at
 * network.PyTorchModel (reference network.py:132-265).  This library sits BELOW
 * a Python class that reproduces that surface (alphazero-gomoku_amd/network.py);
 * each entry point below replaces the ATen work behind one reference call:
 *
 *   azg_pv_forward        <- PyTorchModel.predict            (network.py:168-183)
 *                            = AlphaZeroNet.forward in eval mode (network.py:85-117)
 *                              + F.softmax(dim=1) (network.py:180)
 *   azg_pv_forward_boards <- Gomoku.get_encoded_state (games/gomoku.py:130-150) on every
 *                            queued leaf + predict + p * valid (mcts/new_mcts_alpha.py:
 *                            158-166), from int8 boards
 *   azg_pv_train_backward <- train_batch: zero_grad, train-mode forward, log_softmax,
 *                            KLDiv(batchmean) + MSE, loss.backward()  (network.py:213-222)
 *   azg_pv_train_apply    <- clip_grad_norm_(params, 3.0) + Adam.step()
 *                                                            (network.py:223-224, 161)
 *   azg_pv_create/destroy <- AlphaZeroNet.__init__ shape config (network.py:41-73)
 *
 * Conventions
 *  - All pointers are DEVICE pointers (HIP, gfx950) unless stated; fp32 everywhere.
 *  - Python/torch owns every tensor: parameters, gradients and Adam moments are
 *    flat buffers in nn.Module.parameters() order with torch's own per-tensor
 *    layout (see azg_pv_param_layout); BN running stats are a flat buffer of
 *    [mean(c) | var(c)] per BatchNorm layer in module order.  The handle owns only
 *    its workspace (packed weights, activations, partial sums).
 *  - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); every
 *    entry point is asynchronous on it, does no host sync and no allocation
 *    unless the batch exceeds the workspace high-water mark.
 *  - Return value: 0 = ok, nonzero = error; azg_pv_last_error() gives the text
 *    (thread-local).  No C++ exception crosses the ABI.
 *  - One handle per process/GPU; not re-entrant (the reference host is
 *    single-threaded too).
 */
#ifndef AZG_PV_H
#define AZG_PV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct azg_pv azg_pv;

typedef struct {
    int32_t blocks;    /* residual blocks (reference default 3; BASELINE 6; Pente 10) */
    int32_t channels;  /* 64, 128 or 256 */
    int32_t board;     /* 15 (only 15x15 is built) */
    int32_t in_ch;     /* 3 input planes */
} azg_pv_config;

/* Version of this ABI (bumped on incompatible change). */
int32_t azg_pv_abi_version(void);

const char* azg_pv_last_error(void);

int32_t azg_pv_create(const azg_pv_config* cfg, azg_pv** out);
int32_t azg_pv_destroy(azg_pv* h);

/* Number of trainable parameters (flat length) and of BN running-stat floats. */
int64_t azg_pv_param_count(const azg_pv* h);
int64_t azg_pv_bn_count(const azg_pv* h);
int32_t azg_pv_num_param_tensors(const azg_pv* h);
/* HOST arrays of length azg_pv_num_param_tensors: element offset and numel of each
 * parameter tensor inside the flat buffer, in nn.Module.parameters() order. */
int32_t azg_pv_param_layout(const azg_pv* h, int64_t* offsets, int64_t* numels);

/* Bind torch-owned flat buffers.  params: azg_pv_param_count floats; grads:
 * azg_pv_grad_count floats = the parameter gradients followed by ONE skip word
 * (ABI 3): azg_pv_train_backward writes 1.0 there when its split-fp16 forward (key 49)
 * met an activation beyond fp16's range, else 0.0; a data-parallel caller all-reduces
 * the whole buffer (any nonzero result skips the step on every rank) and
 * azg_pv_train_apply commits the step only where the word is 0.  bn_stats:
 * azg_pv_bn_count floats.  grads may be NULL for inference-only use. */
int32_t azg_pv_bind(azg_pv* h, float* params, float* grads, float* bn_stats);
int64_t azg_pv_grad_count(const azg_pv* h);

/* Optional: bind the int64 num_batches_tracked counters, one per BatchNorm layer
 * in module order (azg_pv_num_bn_layers of them, device).  Each
 * azg_pv_train_backward then advances all of them by one inside its own kernels
 * (the train-mode forward's update, network.py:213 via nn.BatchNorm2d). */
int32_t azg_pv_bind_counters(azg_pv* h, int64_t* num_batches_tracked);
int32_t azg_pv_num_bn_layers(const azg_pv* h);

/* Parameters or BN stats changed outside the library (load_state_dict, copy_, a
 * write through the bound pointers, a collective that rewrites them): re-derive
 * packed weights / folded BN before the next forward AND the next train step.
 * azg_pv_train_apply refreshes the packs itself; between two train steps the
 * library trusts them unless this is called (the Python engine calls it whenever a
 * parameter tensor's version counter moved). */
int32_t azg_pv_mark_dirty(azg_pv* h);

/* Eval-mode forward (BN running stats).  x: [batch,3,15,15] NCHW fp32.
 * probs: [batch,225] softmax(logits); values: [batch,1] tanh; logits: optional
 * [batch,225] (NULL to skip). */
int32_t azg_pv_forward(azg_pv* h, const float* x, int32_t batch,
                       float* probs, float* values, float* logits, void* stream);

/* Eval-mode forward from int8 boards: boards [batch,225] (0 empty, 1, 2), players
 * [batch] (side to move, 1|2), both device.  The reference encoding (planes
 * board==player, board==3-player, ones) is built inside the stem kernel.  probs /
 * values as azg_pv_forward; priors (optional, NULL to skip): probs * (board == 0),
 * the reference's masked prior, bitwise equal to numpy's p * valid. */
int32_t azg_pv_forward_boards(azg_pv* h, const int8_t* boards, const int8_t* players, int32_t batch,
                              float* probs, float* values, float* priors, void* stream);

/* Train-mode forward + loss + backward on the local batch (reference
 * network.py:213-222).  Writes d(loss)/d(param) into the bound grad buffer
 * (overwrites: zero_grad semantics), updates BN running stats (momentum 0.1,
 * unbiased var), and writes {policy_loss, value_loss, total_loss} as 3 floats
 * to losses (device).  pis: [batch,225]; zs: [batch,1]. */
int32_t azg_pv_train_backward(azg_pv* h, const float* x, const float* pis,
                              const float* zs, int32_t batch, float* losses,
                              void* stream);

/* clip_grad_norm_(max_norm) over the bound grads (call after any DP all-reduce
 * of the grad buffer), then one Adam step (torch semantics: L2-coupled weight
 * decay, bias correction for `step`, which is the post-increment step count).
 * exp_avg / exp_avg_sq: flat buffers like params.  total_norm (device, 1 float,
 * may be NULL) receives the pre-clip global L2 norm.
 * If the grad buffer's skip word (azg_pv_bind) is nonzero the step does NOT commit:
 * params, grads and moments are left as they are, the BN running stats and counters
 * are restored to what the step started from, and the skipped-step count
 * (azg_pv_train_status) advances.  The caller then redoes the step, e.g. after
 * azg_pv_train_fp32_once, with the same `step`. */
int32_t azg_pv_train_apply(azg_pv* h, float* exp_avg, float* exp_avg_sq,
                           int64_t step, float lr, float beta1, float beta2,
                           float eps, float weight_decay, float max_norm,
                           float* total_norm, void* stream);

/* The next azg_pv_train_backward on this handle runs its forward convs with fp32
 * MFMA (tuning key 49 = 0 for that one step): the redo of a skipped step. */
int32_t azg_pv_train_fp32_once(azg_pv* h);

/* Kernel-class event timing (bench / roofline instrumentation).  When enabled,
 * every launch of a profiled class is bracketed by hipEvents on the stream it is
 * launched on; azg_pv_profile_read synchronises those events and returns the
 * summed device time (ms) and launch count per class since the last enable. */
enum {
    AZG_PROF_CONV3X3 = 0,   /* residual 3x3 conv, eval epilogue        */
    AZG_PROF_STEM = 1,
    AZG_PROF_HEADS = 2,
    AZG_PROF_TRAIN_CONV = 3, /* train-mode 3x3 conv fwd + dgrad        */
    AZG_PROF_TRAIN_WGRAD = 4,
    AZG_PROF_TRAIN_OTHER = 5,
    AZG_PROF_TOWER = 6,      /* persistent residual tower (all 2*NB convs, one launch),
                                64x64 / 128x64 tiles, 2-4 workgroups per CU          */
    AZG_PROF_TOWER_WIDE = 7, /* the same with 128x128 tiles: 16 waves, 1 workgroup per CU
                                (fp32), or h3_tile's 4 waves of 64x64 (split-fp16, shape 12) */
    AZG_PROF_BOARD = 8,      /* the board-resident tower (split-fp16, C = 128, shape 13): one
                                board's activations in LDS through all 2*NB convs */
    AZG_PROF_BOARD16 = 9,    /* the 16x16x32 board tower (key 19 = 2, C = 128) */
    AZG_PROF_NCLASS = 10
};
int32_t azg_pv_profile_enable(azg_pv* h, int32_t enable);
int32_t azg_pv_profile_read(azg_pv* h, double* ms, int64_t* launches);
/* Boards (eval) / samples (train) processed per class since the last enable, so a
 * caller can price launches of varying batch (self-play) in algorithmic FLOPs.
 * A residual-conv launch (CONV3X3) counts its batch once per conv; a TOWER / TOWER_WIDE /
 * BOARD launch counts its batch once for all 2*blocks convs. */
int32_t azg_pv_profile_boards(const azg_pv* h, int64_t* boards);

/* Process-wide tuning knobs (benchmarks / A-B tests).  Returns the previous value.
 *   key 0: force the 3x3-conv tile shape index (-1 = automatic);
 *   key 1: conv autotuning on/off (default on: the first launch for a (C, M) times
 *          every tile shape on the real operands and caches the fastest; shapes give
 *          bitwise-identical results, so this never changes numerics);
 *   key 2: query the tuned shape for value = M*1024 + C (-1 if not tuned yet);
 *   key 4: conv kernel variant (1 halo-staged, default; 0 per-chunk staging, timing only);
 *   key 5: eval residual tower: 0 one launch per conv, 1 one persistent launch
 *          (shape from key 6), 2 (default) chosen per (C, blocks, batch bucket) by
 *          timing every variant on first use -- all bitwise identical;
 *   key 6: persistent-tower tile shape for key 5 = 1 (8: 128x64 / 8 waves, default;
 *          5: 64x64 / 4 waves; 10: 128x128 / 16 waves, one workgroup per CU, C = 128, fp32
 *          only; 12: h3_tile 128x128 / 4 waves of 64x64, split-fp16 only; 13: the
 *          board-resident tower (pv_board.hip: one board per 16-wave workgroup, its
 *          activations in LDS through every conv), split-fp16 and C = 128 only -- a shape
 *          the current arithmetic lacks runs as 8); with key 19 = 2 at C = 128 keys 5 / 6
 *          do not apply (one form: the 16x16x32 board tower);
 *   keys 3, 7, 8: timing-only ablation switches (results invalid while set);
 *   key 10: tile-body variant of the C=128 128x64 persistent tower (0 = default;
 *          1..5 = swizzle / prefetch / LDS-DMA staging variants for A/B timing, all
 *          bitwise identical to 0);
 *   key 9: stem kernel (1 = fp32 MFMA, default; 0 = VALU reference, bitwise equal);
 *   key 11: stem ablation mask (timing only, results invalid while set);
 *   key 17: persistent-tower claim granularity (1 = one M tile with all its N
 *          tiles, run back to back by the claiming workgroup, default: the second
 *          tile's halo rows hit the XCD's L2, +2 % at B = 512 and 4096, measured;
 *          0 = one 128x64 tile per claim); bitwise identical results;
 *   key 21: per-layer 128x64 conv: the last partial round of workgroups runs as a
 *          second launch of 64x64 tiles (1, default) or not (0); bitwise identical;
 *   key 22: per-layer 128x64 conv tile body (1 = halo rows keyed on the board
 *          position, conflict-free fragment reads, default; 0 = row-keyed; 4 / 5 =
 *          LDS-DMA staging); bitwise identical;
 *   key 23: train forward BN apply + ReLU (+ residual) folded into the next conv's
 *          halo staging (1, default; C <= 128 only: at C = 256 the prologue spills
 *          and the separate passes are faster) or separate bn_apply passes (0);
 *          bitwise identical;
 *   key 24: train BN finalize run by the last workgroup of the conv producing the
 *          layer's partials (1, default) or by separate finalize kernels (0); one
 *          shared fp64 reduction order, bitwise identical;
 *   key 27: train conv weight-grad pixel splits (0 = automatic, default; 8..64, a
 *          multiple of 8); bitwise identical only at a fixed value;
 *   key 44: train BN apply / BN-backward apply passes: workgroup cap of their
 *          grid-stride launch (0 = four float4 per thread, default); bitwise identical;
 *   key 31: study build only: the 64x64 / 128x64 towers with sc1 dependent loads
 *          and no acquire (two or more workgroups per CU: outside the microarch
 *          guide's measured envelope; the product uses the acquire there and the
 *          sc1 form only for the one-workgroup-per-CU 16-wave tile); returns 0 in
 *          the product library;
 *   key 14: persistent-tower dependency wait bound in microseconds of the waiting
 *          wave's awake time (default 100000 = 100 ms; -1 restores it; 0 makes every
 *          dependency wait time out at once, exercising the recovery path);
 *   key 19: eval residual-conv arithmetic: 2 (default) and 1 split-fp16 -- every fp32
 *          operand x is split into hi = fp16(x), lo = fp16(x - hi) and a product is lo*hi +
 *          hi*lo + hi*hi by fp16 MFMAs with fp32 accumulation (weights scaled by a per-layer
 *          power of two, undone in the BN scale; error ~2^-22 per product, the fp32 MFMA
 *          chain's order of magnitude); 1 sums 16 channels per
 *          v_mfma_f32_32x32x16_f16 (per-layer launches, tile towers, the 32x32 board
 *          tower), 2 at C = 128 sums 32 per v_mfma_f32_16x16x32_f16 in the 16x16x32 board
 *          tower (pv_board16.hip), the one form of that arithmetic (C = 256: as 1); 0 fp32
 *          MFMA.  Every eval path (tower, per-layer, recompute) uses the selected
 *          arithmetic, so within it the forms are bitwise equal and the forward is
 *          batch-independent.  An activation at or above fp16's
 *          range (65520 rounds to inf) makes its products non-finite: the epilogue posts
 *          the launch and azg_pv_recover recomputes it with fp32 MFMA.  The train step
 *          always uses fp32 MFMA;
 *   key 52: key 19 = 2 at C = 128: the largest batch whose boards each run over three 8-wave
 *          workgroups (pixel thirds) that exchange their conv outputs' 16 boundary rows through
 *          L2 (default 85: 3 x 85 workgroups fit 256 CUs; 0 never) -- bitwise the one-workgroup
 *          tower, about 2/3 of its latency; a timed-out exchange wait (key 14) posts the launch
 *          (azg_pv_recover reruns it one workgroup per board);
 *   key 20: the split-fp16 tower's tile body (1 = halo rows keyed on the board position,
 *          conflict-free fragment reads, default; 0 = row-keyed); bitwise identical;
 *   key 49: train-step forward convs: 2 (default) split-fp16 with all four hi / lo products
 *          (~2^-33 per product: the two-step goldens hold), 1 three products, 0 fp32 MFMA;
 *          the dgrad convs and weight grads stay fp32; a staged activation beyond fp16's
 *          range sets the step's skip word (azg_pv_bind): the step does not commit and the
 *          caller redoes it in fp32 (azg_pv_train_fp32_once);
 *   key 48: train weight-grad tile (1 = padded-row table, buffer LDS-DMA, slabs in the
 *          MFMA layout, default; 0 = round-4 form); bitwise identical;
 *   key 18: seconds a handle runs per-layer convs after azg_pv_recover recomputed one
 *          of its tower launches (default 30; 0 disables the breaker).  A timed-out
 *          wait means parts of the dispatch were suspended while others ran (the GPU is
 *          shared with another process); per-layer launches have no
 *          cross-workgroup waits.
 *   Every call returns the previous value. */
int32_t azg_pv_set_tuning(int32_t key, int32_t value);

/* Persistent-tower dependency waits (pv_tower.hip).  A tile of the one-launch eval
 * tower waits for the three tiles of the previous layer whose rows its halo reads.
 * The wait is bounded by the waiting wave's AWAKE time (s_memrealtime deltas, each
 * capped at 10 us, so a wave that was suspended together with its producer resumes
 * without timing out); past the bound (key 14) the tile computes on stale inputs, the
 * launch drains, and the launch's sequence number is posted to a ring in pinned,
 * mapped host memory.  Every forward that runs the tower gets a sequence number
 * (azg_pv_last_seq: the last one on this handle, 0 if the last forward ran per-layer
 * convs).  azg_pv_recover(seq) -- called after synchronising with that forward --
 * recomputes a posted launch with per-layer convs (bitwise equal to a tower that did
 * not time out) into the SAME output buffers on `stream`, provided the caller's input
 * and output buffers of that forward are still intact; *recovered = 1 then (0: the
 * launch did not time out).  The Python layer does this at every host-synchronising
 * forward (predict, predict_boards, BoardEvaluator.wait), so a timeout costs one
 * per-layer forward instead of an error. */
/* Error word of the last tower launch on this handle: 1 if one of its waits timed
 * out (synchronises `stream`). */
int32_t azg_pv_tower_status(azg_pv* h, void* stream);
uint32_t azg_pv_last_seq(const azg_pv* h);
int32_t azg_pv_recover(azg_pv* h, uint32_t seq, int32_t* recovered, void* stream);

/* Number of posted eval launches not yet recovered -- timed-out tower launches and
 * split-fp16 launches whose activations left fp16's range (a plain host load of the
 * pinned rings: complete for every forward the caller has synchronised with).
 * azg_pv_posted(seq): bit 0 = launch `seq` timed out, bit 1 = it met a range overflow,
 * both not yet recovered (0: nothing to settle).  The Python layer raises on a posted
 * launch it cannot recover (its buffers are gone).  azg_pv_clear_status drops every
 * posted launch without recomputing it, zeroes the skipped-step count and closes the
 * per-layer breaker (key 18). */
int32_t azg_pv_status(const azg_pv* h);
int32_t azg_pv_posted(const azg_pv* h, uint32_t seq);
int32_t azg_pv_clear_status(azg_pv* h);
/* Train steps azg_pv_train_apply skipped because their skip word was set (a split-fp16
 * train forward, key 49, met an activation beyond fp16's range on some rank) since the
 * last azg_pv_clear_status (a plain host load; complete for every step the caller has
 * synchronised with). */
int32_t azg_pv_train_status(const azg_pv* h);

/* Self-describing record of the tower's waits since the last azg_pv_tower_diag_clear
 * (device counters + the first timed-out wait; synchronises `stream`).  Times are
 * microseconds from s_memrealtime (100 MHz).  hwid = the HW_ID hardware register of the
 * wave (CU, SE, VMID, queue, ...), xcc = its XCD (HW_REG_XCC_ID). */
typedef struct {
    uint32_t timeouts;          /* waits that timed out */
    uint32_t waits_over_100us;  /* waits whose awake time exceeded 0.1 / 1 / 10 / 100 ms */
    uint32_t waits_over_1ms;
    uint32_t waits_over_10ms;
    uint32_t waits_over_100ms;
    uint32_t max_wait_us;       /* longest awake wait */
    uint32_t recovered;         /* launches recomputed by azg_pv_recover (host count) */
    /* the first timed-out wait */
    uint32_t seq;               /* its launch */
    uint32_t layer;             /* the waiting tile: conv layer (1 .. 2*blocks-1) and M tile */
    uint32_t mtile;
    uint32_t wait_mtile;        /* the layer-1 M tile it waited on */
    uint32_t observed;          /* that tile's completion counter when the wait gave up */
    uint32_t needed;            /* ... and the value it waited for (N tiles per M tile) */
    uint32_t waited_us;         /* awake time of the wait */
    uint32_t wall_us;           /* wall time from the wait's start to its timeout */
    uint32_t waiter_hwid, waiter_xcc;
    uint32_t claims;            /* tiles claimed in the launch when it timed out */
    uint32_t producer_claimed;  /* 1: the producer tile had been claimed */
    uint32_t producer_started;  /* 1: its workgroup had started it in this launch */
    uint32_t producer_hwid, producer_xcc;
    int32_t producer_start_us;  /* its start relative to the wait's start */
    uint32_t max_wall_us;       /* longest WALL time of a wait (awake + suspended) */
    uint32_t waits_suspended;   /* waits whose wall time exceeded their awake time by > 1 ms */
    uint32_t breaker_trips;     /* recoveries that switched the handle to per-layer convs (key 18) */
    uint32_t breaker_launches;  /* forwards run per layer while the breaker was open */
    uint32_t h3_overflows;      /* split-fp16 forwards recomputed with fp32 MFMA (key 19: an activation
                                   beyond fp16's range, 65504) */
    uint32_t train_h3_overflows;   /* train steps skipped because a split-fp16 train forward (key 49) met an
                                      activation beyond fp16's range (= azg_pv_train_status; the Python layer
                                      redoes each in fp32; azg_pv_clear_status resets it) */
    uint32_t reserved[3];
} azg_pv_tower_diag;
int32_t azg_pv_tower_diag_read(azg_pv* h, azg_pv_tower_diag* out, void* stream);
int32_t azg_pv_tower_diag_clear(azg_pv* h, void* stream);

/* Debug/test access to train-workspace activations of the last train step:
 * copies the interior [batch][15][15][C] (NHWC) of buffer `which` (block `index`
 * where relevant) into dst (device, batch*225*C floats), stream-ordered.
 * which: 0 z0 (stem conv out), 1 a0 (stem act), 2 z1[i], 3 h[i], 4 z2[i],
 * 5 xo[i] (block out), 6 gX, 7 DZ, 8 DH, 9 GR, 10 gX snapshot i (env
 * AZG_DEBUG_SNAP), and raw head features (no unpadding): 11 policy features
 * [batch][450], 12 value features [batch][225], 13 value hidden [batch][64]. */
int32_t azg_pv_debug_copy(azg_pv* h, int32_t which, int32_t index, float* dst,
                          int32_t batch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AZG_PV_H */
