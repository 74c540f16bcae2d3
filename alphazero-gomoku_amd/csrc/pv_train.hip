// Train step (placeholder until the training kernels land).
#include "pv_internal.h"

namespace azg {
void free_train_workspace(azg_pv* h) { (void)h; }
}  // namespace azg

extern "C" int32_t azg_pv_train_backward(azg_pv* h, const float* x, const float* pis, const float* zs,
                                         int32_t batch, float* losses, void* stream)
{
    (void)h; (void)x; (void)pis; (void)zs; (void)batch; (void)losses; (void)stream;
    return azg::set_error("azg_pv_train_backward: not built yet", hipSuccess);
}

extern "C" int32_t azg_pv_train_apply(azg_pv* h, float* exp_avg, float* exp_avg_sq, int64_t step, float lr,
                                      float beta1, float beta2, float eps, float weight_decay, float max_norm,
                                      float* total_norm, void* stream)
{
    (void)h; (void)exp_avg; (void)exp_avg_sq; (void)step; (void)lr; (void)beta1; (void)beta2; (void)eps;
    (void)weight_decay; (void)max_norm; (void)total_norm; (void)stream;
    return azg::set_error("azg_pv_train_apply: not built yet", hipSuccess);
}
