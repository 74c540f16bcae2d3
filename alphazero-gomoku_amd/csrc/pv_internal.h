// Internal (non-ABI) declarations shared by the C-ABI and the kernel launchers.
#pragma once
#include "pv_common.h"
#include "../../include/azg_pv.h"

#include <vector>

namespace azg {

struct BnDesc {
    int gamma_off;
    int beta_off;
    int stat_off;
    int c;
    int out_off;
    int pad[3];
};

struct BlockTensors { int w1, g1, b1, w2, g2, b2; };

// strided fp32 GEMM problem (pv_gemm.hip): C(i,j) = sum_k A(i,k) B(k,j), optionally
// zeroed where mask(i,j) <= 0
struct GemmProb {
    const float* A; int sai, sak;
    const float* B; int sbk, sbj;
    float* C; int sci, scj;
    const float* mask; int smi, smj;
    int M, N, K;
};
struct GemmPair { GemmProb p[2]; int ntn0; };
struct BlockBn { int first, second; };

// kernel launchers (pv_conv.hip, pv_heads.hip, pv_pack.hip, pv_train.hip)
hipError_t launch_conv3x3(int C, int epi, const float* in, const float* wp, const float* scale,
                          const float* shift, const float* resid, float* out, int M, hipStream_t st);
struct EpiX;
struct ProX;
struct FinX;
constexpr int TRAIN_BM = 128;   // rows per M tile of conv3x3_train (BN partials granularity)
// oscale (forward convs only): the split-fp16 weights of pack_h3 are passed as wp and the
// raw output is multiplied by oscale[c] (= 2^-e of the layer, exact); nullptr: fp32 weights
hipError_t launch_conv3x3_train(int C, int epi, int xe, const float* in, const float* wp, const float* resid,
                                float* out, int M, const EpiX& ex, hipStream_t st, const ProX* px = nullptr,
                                const FinX* fx = nullptr, const float* oscale = nullptr, unsigned* h3ovf = nullptr,
                                const unsigned* dmax = nullptr);
extern int g_train_dgrad_h3;   // key 50: the train step's dgrad convs in split-fp16 (2: four products, 1: three, 0: fp32)
extern int g_train_h3;   // key 49: the train step's forward convs in split-fp16 (1) or fp32 MFMA (0)
extern int g_tower_mode;
extern int g_conv_shape_override;
extern int g_tower_shape;
extern int g_tower_ablation;
extern int g_tower_var;
extern int g_train_fuse_apply;
extern int g_train_fuse_fin;
extern int g_train_apply_grid;
extern int g_wgrad_splits;
extern int g_wgrad_variant;
hipError_t launch_stem_stats(int C, const float* x, const float* ws, float* out, int B, float* pa, float* pb,
                             hipStream_t st);
constexpr int kTowerMaxBlocks = 32;
int conv_batch_bucket(int M);
size_t tower_sync_bytes(int nlayers, int M);
size_t tower_prod_bytes(int nlayers, int M);
constexpr unsigned kTowerRing = 256;          // host ring of timed-out launch numbers (power of 2)
constexpr unsigned kTrainOvfWords = 16;       // + the train step's words (same memory): [kTrainFlag] the split-fp16
                                              // train forward's overflow flag of the step in flight (moved into the
                                              // gradient buffer's skip slot and cleared by heads_small_grads),
                                              // [kTrainSkips] steps the Adam kernel skipped (azg_pv_train_status)
constexpr unsigned kTrainFlag = 1, kTrainSkips = 2;
constexpr unsigned kStatusWords = 2 * kTowerRing + kTrainOvfWords;
constexpr int kTowerDiagWords = 64;           // device wait record (pv_tower.hip TowerDiag)
constexpr unsigned kTowerWaitUs = 100000u;    // default awake-time bound of one dependency wait: 100 ms
                                              // (longest legitimate wait measured: 7.3 ms, two processes
                                              // sharing the GPU; 0.26 ms alone -- DESIGN.md section 7)
extern int g_tower_breaker_s;                 // key 18: seconds of per-layer convs after a recovered launch
struct TowerSync {
    unsigned* sync;   // tower_sync_bytes: memset per launch
    unsigned* ring;   // host-mapped ring (device alias)
    unsigned* ring_ovf;   // host-mapped ring of H3 range overflows (device alias)
    unsigned* diag;   // kTowerDiagWords, persistent
    void* prod;       // tower_prod_bytes, persistent
    unsigned seq;     // launch number (0: not posted)
};
hipError_t launch_tower(int C, int NB, int shape, float* const act[3], const float* wpack, const float* scale,
                        const float* shift, const int* out_off, int M, const TowerSync& ts, hipStream_t st,
                        float** result, bool h3 = false);
// board-resident split-fp16 tower (pv_board.hip, C = 128): x = the stem output, overwritten in
// place with the tower output
hipError_t launch_board_tower(int NB, const float* wp16, const float* scale16, const float* shift, const int* out_off,
                              float* x, int B, unsigned* ring_ovf, unsigned seq, hipStream_t st);
// small batches (B <= key 52, 3 B <= CUs): each board over three workgroups that exchange conv
// outputs' boundary rows through `xbuf` (bitwise the one-workgroup tower); hout must be null
struct Board16Split {
    char* xbuf;        // [B][2][4 * 226 * 128 B] exchange images (zero rows: zero)
    unsigned* xflag;   // [B][3] publish flags (monotonic over launches: tags epoch * 64 + layer + 1)
    unsigned epoch;    // > every earlier split launch's on these flags
    unsigned* ring;    // timed-out launch ring (device alias), azg_pv_recover
    unsigned* diag;    // the tower wait record
};
extern int g_board16_split;   // key 52
int board16_grid();           // workgroups of a one-per-CU board16 launch (0: init failed)
int board16_split_max();      // largest batch the split form takes (key 52, CUs / 3, kB16SplitCap)
constexpr int kB16SplitCap = 85;                        // 3 x 85 workgroups <= 256 CUs
constexpr size_t kB16ImgBytes = 4 * (15 * 15 + 1) * 128;   // pv_board16.hip kB16Img
// hout != nullptr: the tower output stays in LDS and the kernel writes the heads' projected
// features (heads_project's, bitwise) to hout [B][FC_FS] instead of x
hipError_t launch_board16_tower(int NB, const float* wp16, const float* scale16, const float* shift,
                                const int* out_off, float* x, int B, unsigned* ring_ovf, unsigned seq, hipStream_t st,
                                const float* hwp = nullptr, const float* hwv = nullptr, const float* hsc = nullptr,
                                const float* hsh = nullptr, float* hout = nullptr, const Board16Split* sp = nullptr);

// the heads' 1x1 projection epilogue: folded eval BN + ReLU (heads_project and the board16 tower)
__device__ __forceinline__ float head_bn_relu(float d, float s, float h) { return fmaxf(d * s + h, 0.f); }
extern unsigned g_tower_wait_us;
extern int g_tower_group;
#ifdef AZG_AB_STUDIES
extern int g_tower_coh;
#endif
hipError_t launch_stem(int C, int epi, const float* x, const float* ws, const float* scale,
                       const float* shift, float* out, int B, hipStream_t st, const int8_t* boards = nullptr,
                       const int8_t* players = nullptr);
hipError_t launch_heads_fwd(int C, const float* act, const float* wpc, const float* wvc,
                            const float* hscale, const float* hshift, const float* wfc,
                            const float* bpf, const float* bv1,
                            const float* wv2, const float* bv2, float* hbuf, float* probs,
                            float* values, float* logits, int B, hipStream_t st,
                            const int8_t* boards = nullptr, float* priors = nullptr, bool projected = false);
hipError_t launch_heads_fc(const float* feat, const float* wfc, float* pre, int B, hipStream_t st);
hipError_t launch_heads_project(int C, bool bn, const float* act, const float* wpc, const float* wvc,
                                const float* hscale, const float* hshift, float* hout, int M, hipStream_t st,
                                int fs = 3 * PIX, int voff = 2 * PIX);
hipError_t launch_pack_fc(const float* wpf, const float* wv1, float* wfc, hipStream_t st);
hipError_t launch_small_gemm(const GemmProb& p0, const GemmProb* p1, hipStream_t st);
hipError_t launch_pack_convs(const float* params, const int64_t* offs, int nl, float* wp, float* wd, int C,
                             hipStream_t st);
hipError_t launch_pack_stem(const float* w, float* ws, int C, hipStream_t st);
hipError_t launch_transpose(const float* src, float* dst, int R, int Cc, hipStream_t st);
hipError_t launch_repack_all(const float* params, const int64_t* conv_offs, int nl, float* wp, float* wd, int C,
                             const float* stem_w, float* ws, const float* wpf, const float* wv1, float* wfc,
                             const float* stats, const void* desc, int nbn, float* scale, float* shift,
                             hipStream_t st, int part = 0);
hipError_t launch_conv3x3_h3(int shape, int C, int epi, const float* in, const float* wp, const float* scale,
                             const float* shift, const float* resid, float* out, int M, hipStream_t st,
                             unsigned* ring, unsigned seq);
hipError_t launch_pack_h3(const float* params, const int64_t* offs, int nl, int C, const int* conv_bn_off,
                          const float* scale, int* exps, void* wp16, float* scale16, float* inv, hipStream_t st);
hipError_t launch_pack_h3_dgrad(const float* params, const int64_t* offs, int nl, int C, const int* exps, void* wd16,
                                hipStream_t st);
extern int g_tower_h3;
extern int g_h3_tower_var;
hipError_t launch_fold_bn(const float* params, const float* stats, const void* desc, int nlayers,
                          float* scale, float* shift, hipStream_t st);

}  // namespace azg

struct azg_pv {
    azg_pv_config cfg{};
    int C = 0, NB = 0;

    // flat layout (nn.Module.parameters() order)
    std::vector<int64_t> poff, pnum;
    int64_t nparams = 0, nbn = 0;
    int nfold = 0;
    int t_stem_w = 0, t_stem_g = 0, t_stem_b = 0;
    std::vector<azg::BlockTensors> t_blk;
    int t_pc_w = 0, t_pbn_g = 0, t_pbn_b = 0, t_pfc_w = 0, t_pfc_b = 0;
    int t_vc_w = 0, t_vbn_g = 0, t_vbn_b = 0, t_vfc1_w = 0, t_vfc1_b = 0, t_vfc2_w = 0, t_vfc2_b = 0;
    std::vector<azg::BnDesc> bn_desc;
    int bn_stem = 0, bn_pol = 0, bn_val = 0;
    std::vector<azg::BlockBn> bn_blk;
    void* bn_desc_dev = nullptr;
    int64_t* conv_off_dev = nullptr;   // flat-param offset of each 3x3 conv weight (2*NB, block order)

    // bound torch-owned buffers
    float* params = nullptr;
    float* grads = nullptr;
    float* bn = nullptr;
    int64_t* nbt = nullptr;   // optional: num_batches_tracked per BN layer (azg_pv_bind_counters)
    bool dirty = true;
    bool train_packs = false;   // wpack / wdpack / wstem / wfc hold the current parameters (train_apply, key 36)
    bool bn_bak_ok = false;     // the train workspace's BN backup holds the running stats the next step starts from
    bool train_fp32_once = false;   // azg_pv_train_fp32_once: the next train step's forward convs in fp32 MFMA

    // packed / derived weights (one allocation)
    float* wbase = nullptr;
    float* wpack = nullptr;   // 2*NB x [9*C/32][C][32]
    float* wstem = nullptr;   // [27][C]
    float* wfc = nullptr;     // [FC_OUT][FC_KP] packed policy_fc + value_fc1 (pv_heads.hip heads_fc)
    float* scale = nullptr;   // folded BN (eval)
    float* shift = nullptr;
    // split-fp16 (H3) eval weights: packed [hi | lo] rows of w * 2^e per conv, the BN
    // scale times 2^-e, the exponents and each conv's BN offset (allocated on first use)
    void* wpack16 = nullptr;
    float* scale16 = nullptr;
    int* h3exp = nullptr;
    float* h3inv = nullptr;   // [2 NB][C]: 2^-e of each conv (train forward, raw outputs)
    int* conv_bn_off_dev = nullptr;
    bool h3_dirty = true;
    unsigned h3_gen = 0;   // + 1 per split-fp16 re-pack (the train step's dgrad pack follows it)

    // eval activations: 3 padded NHWC buffers + head features [B][3][225]
    float* act[3] = {nullptr, nullptr, nullptr};
    float* hbuf = nullptr;
    unsigned* tower_sync = nullptr;   // persistent tower: work counter, error word, tile counters
    void* tower_prod = nullptr;       // persistent tower: per-tile producer records
    unsigned* tower_diag = nullptr;   // persistent tower: wait record (kTowerDiagWords, device)
    unsigned* ring_host = nullptr;    // timed-out launch numbers [kTowerRing], pinned + mapped (kernels post, host reads)
    unsigned* ring_dev = nullptr;     // device alias of ring_host
    unsigned* ovf_host = nullptr;     // H3 launches whose activations left fp16's range [kTowerRing], same memory
    unsigned* train_ovf_dev = nullptr;   // [kTrainOvfWords] split-fp16 train forward overflow flags (device alias)
    unsigned* ovf_dev = nullptr;
    char* b16x = nullptr;             // board16 split exchange images [kB16SplitCap][2][image] (zeroed)
    unsigned* b16flag = nullptr;      // [kB16SplitCap][3] publish flags
    unsigned b16epoch = 0;            // split launches so far (their flag tags)
    bool b16_split = false;           // the last forward's board16 launch ran split (heads unfused)
    unsigned seq = 0;                 // last tower launch number handed out (0 = none yet)
    unsigned last_seq = 0;            // the last forward's launch number (0: it ran per-layer convs)
    // what each posted launch read and wrote, by seq % kTowerRing (azg_pv_recover re-runs it)
    struct LaunchRec {
        unsigned seq = 0;
        const float* x = nullptr;
        const int8_t* boards = nullptr;
        const int8_t* players = nullptr;
        int batch = 0;
        bool h3 = false;
        float *probs = nullptr, *values = nullptr, *logits = nullptr, *priors = nullptr;
    };
    std::vector<LaunchRec> launches;
    uint32_t recovered = 0;           // launches recomputed per layer
    uint32_t h3_overflows = 0;        // H3 launches recomputed with fp32 MFMA (activations beyond fp16's range)
    // circuit breaker: a recovered launch means the dispatch did not run as one (the GPU is
    // shared and parts of it were suspended); forwards run per-layer convs until then
    double breaker_until = 0.0;       // steady-clock seconds
    uint32_t breaker_trips = 0;
    uint32_t breaker_launches = 0;    // forwards that ran per layer because of it
    int act_cap = 0;

    // train workspace (pv_train.hip)
    void* train = nullptr;

    // kernel-class event timing (azg_pv_profile_*)
    bool prof_on = false;
    std::vector<hipEvent_t> prof_ev;     // pairs
    std::vector<int> prof_cls;           // class per used pair
    int prof_used = 0;
    double prof_ms[AZG_PROF_NCLASS] = {};
    int64_t prof_n[AZG_PROF_NCLASS] = {};
    int64_t prof_work[AZG_PROF_NCLASS] = {};   // boards (or samples) processed per class
};

namespace azg {
int32_t set_error(const char* what, hipError_t e);
void build_layout(azg_pv* h);
void free_workspace(azg_pv* h);
void free_train_workspace(azg_pv* h);
int32_t ensure_eval_workspace(azg_pv* h, int batch, hipStream_t st);
int32_t repack(azg_pv* h, hipStream_t st, float* dgrad_dst = nullptr, int part = 0);   // dgrad_dst: also pack dgrad weights
int32_t ensure_h3(azg_pv* h, hipStream_t st);   // split-fp16 packs of the current parameters
int prof_begin(azg_pv* h, int cls, hipStream_t st, int64_t boards = 0);   // returns pair index or -1
hipError_t prof_harvest(azg_pv* h);
void prof_end(azg_pv* h, int pair, hipStream_t st);
int32_t forward_eval(azg_pv* h, const float* x, int batch, float* probs, float* values, float* logits,
                     hipStream_t st, const int8_t* boards, const int8_t* players, float* priors,
                     bool per_layer = false, bool fp32_only = false, unsigned guard_seq = 0);
}  // namespace azg
