// Host AddressSanitizer driver of the policy/value C-ABI's host side
// (include/azg_pv.h, csrc/pv_capi.hip built with -Xarch_host -fsanitize=address):
// handle lifecycle, flat-buffer layout for every supported shape, the status and
// tuning entry points, and every argument-error path.  No kernel runs (the driver
// also works without a GPU: device work is only reached after azg_pv_bind).
#include "../../../include/azg_pv.h"

#include <cstdio>
#include <cstring>
#include <vector>

static int fails = 0;
#define CHECK(c)                                                                          \
    do {                                                                                  \
        if (!(c)) {                                                                       \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            ++fails;                                                                      \
        }                                                                                 \
    } while (0)

int main()
{
    CHECK(azg_pv_abi_version() == 3);
    const int shapes[4][2] = {{3, 64}, {6, 128}, {10, 256}, {0, 64}};
    const long long want[3] = {340010, 1892650, 11930922};
    for (int s = 0; s < 4; ++s) {
        azg_pv_config cfg{shapes[s][0], shapes[s][1], 15, 3};
        azg_pv* h = nullptr;
        CHECK(azg_pv_create(&cfg, &h) == 0 && h);
        const int64_t n = azg_pv_param_count(h);
        if (s < 3) CHECK(n == want[s]);
        CHECK(azg_pv_grad_count(h) == n + 1);   // + the step's skip word (ABI 3)
        const int nt = azg_pv_num_param_tensors(h);
        std::vector<int64_t> off(nt), num(nt);
        CHECK(azg_pv_param_layout(h, off.data(), num.data()) == 0);
        int64_t o = 0;
        for (int i = 0; i < nt; ++i) {
            CHECK(off[i] == o);
            o += num[i];
        }
        CHECK(o == n);
        CHECK(azg_pv_bn_count(h) > 0 && azg_pv_num_bn_layers(h) == 2 * shapes[s][0] + 3);
        CHECK(azg_pv_status(h) == 0);
        CHECK(azg_pv_train_status(h) == 0);
        CHECK(azg_pv_clear_status(h) == 0);
        CHECK(azg_pv_mark_dirty(h) == 0);
        // tower recovery / wait record before any launch: nothing posted, nothing to do
        CHECK(azg_pv_last_seq(h) == 0);
        CHECK(azg_pv_posted(h, 0) == 0 && azg_pv_posted(h, 7) == 0);
        CHECK(azg_pv_train_fp32_once(h) == 0);
        int32_t rec = -1;
        CHECK(azg_pv_recover(h, 0, &rec, nullptr) == 0 && rec == 0);
        CHECK(azg_pv_recover(h, 7, &rec, nullptr) == 0 && rec == 0);
        CHECK(azg_pv_recover(h, 7, nullptr, nullptr) != 0);
        azg_pv_tower_diag d;
        std::memset(&d, 0xff, sizeof(d));
        CHECK(azg_pv_tower_diag_read(h, &d, nullptr) == 0 && d.timeouts == 0 && d.recovered == 0);
        CHECK(azg_pv_tower_diag_read(h, nullptr, nullptr) != 0);
        CHECK(azg_pv_tower_diag_clear(h, nullptr) == 0);
        // not bound yet: every compute entry point must fail cleanly
        float dummy = 0.f;
        CHECK(azg_pv_forward(h, &dummy, 1, &dummy, &dummy, nullptr, nullptr) != 0);
        CHECK(std::strlen(azg_pv_last_error()) > 0);
        CHECK(azg_pv_forward_boards(h, nullptr, nullptr, 1, &dummy, &dummy, nullptr, nullptr) != 0);
        CHECK(azg_pv_train_backward(h, &dummy, &dummy, &dummy, 4, &dummy, nullptr) != 0);
        CHECK(azg_pv_train_apply(h, &dummy, &dummy, 1, 1e-3f, 0.9f, 0.999f, 1e-8f, 1e-4f, 3.f, nullptr, nullptr) != 0);
        CHECK(azg_pv_destroy(h) == 0);
    }
    // invalid configurations
    azg_pv* h = nullptr;
    azg_pv_config bad1{6, 96, 15, 3}, bad2{6, 128, 19, 3}, bad3{6, 128, 15, 4}, bad4{-1, 64, 15, 3};
    CHECK(azg_pv_create(&bad1, &h) != 0 && h == nullptr);
    CHECK(azg_pv_create(&bad2, &h) != 0);
    CHECK(azg_pv_create(&bad3, &h) != 0);
    CHECK(azg_pv_create(&bad4, &h) != 0);
    CHECK(azg_pv_create(nullptr, &h) != 0);
    CHECK(azg_pv_destroy(nullptr) == 0);
    CHECK(azg_pv_param_count(nullptr) == -1);
    CHECK(azg_pv_status(nullptr) == 0);
    CHECK(azg_pv_train_status(nullptr) == 0);
    CHECK(azg_pv_posted(nullptr, 3) == 0);
    CHECK(azg_pv_grad_count(nullptr) == -1);
    CHECK(azg_pv_train_fp32_once(nullptr) != 0);
    CHECK(azg_pv_last_seq(nullptr) == 0);
    CHECK(azg_pv_tower_diag_clear(nullptr, nullptr) != 0);
    CHECK(azg_pv_bind(nullptr, nullptr, nullptr, nullptr) != 0);
    // tuning keys round-trip (previous value returned)
    const int prev = azg_pv_set_tuning(5, 0);
    CHECK(azg_pv_set_tuning(5, prev) == 0);
    CHECK(azg_pv_set_tuning(999, 1) == -1);
    const int prev_wait = azg_pv_set_tuning(14, 0);   // wait bound (us): default 1 s
    CHECK(prev_wait == 100000);
    CHECK(azg_pv_set_tuning(14, -1) == 0 && azg_pv_set_tuning(14, -1) == 100000);
    const int prev_breaker = azg_pv_set_tuning(18, 0);   // breaker seconds: default 30
    CHECK(prev_breaker == 30 && azg_pv_set_tuning(18, prev_breaker) == 0);
    std::printf("asan_pv: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
