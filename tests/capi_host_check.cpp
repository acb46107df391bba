// Host-only driver of the C-ABI's argument validation, built against the AddressSanitizer objects of the
// library (marl-sat_amd/Makefile `debug`: -Xarch_host -fsanitize=address) and run on the CPU by
// tests/test_debug_build.py.  Every call below must be rejected by the host glue before anything reaches
// the GPU (there is none in the build container): the calls exercise the validation branches, the
// thread-local error channel (vsnprintf into msat_last_error's buffer) and the plan arithmetic under ASan.
// Exit 0 when every check holds; otherwise the failing check is printed and the exit code is 1.
#include <stdio.h>
#include <string.h>

#include "marlsat.h"
#include "marlsat_net.h"

static int g_fail = 0;

static void expect(int rc, int want, const char *needle, const char *what) {
    const char *msg = msat_last_error();
    if (rc != want || (needle && !strstr(msg, needle))) {
        printf("FAIL %s: rc %d (want %d), message '%s' (want '%s')\n", what, rc, want, msg, needle ? needle : "");
        g_fail = 1;
    }
}

int main() {
    msat_env_desc d;
    memset(&d, 0, sizeof(d));
    d.num_envs = 4;
    d.num_vars = 20;
    d.num_clauses = 91;
    d.clause_width = 3;
    d.num_agents = 2;
    d.max_vars_per_agent = 10;
    d.max_steps = 512;
    d.num_problems = 1;
    msat_pool pool = {nullptr, nullptr, nullptr};
    msat_env_state st;
    memset(&st, 0, sizeof(st));
    msat_step_out out;
    memset(&out, 0, sizeof(out));

    // env boundary (marlsat.h)
    msat_env_desc bad = d;
    bad.num_vars = 0;
    expect(msat_env_step(&bad, &pool, &st, nullptr, 0, nullptr, nullptr, 0, 0, &out, nullptr, nullptr), MSAT_EBADARG,
           "num_vars", "env_step num_vars");
    bad = d;
    bad.clause_width = 4;
    expect(msat_env_reset(&bad, &pool, &st, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr), MSAT_EBADARG,
           "clause_width", "env_reset clause_width");
    expect(msat_env_step(&d, &pool, &st, nullptr, 0, nullptr, nullptr, 0, 0, &out, nullptr, nullptr), MSAT_EBADARG,
           nullptr, "env_step NULL state");
    expect(msat_env_step(nullptr, &pool, &st, nullptr, 0, nullptr, nullptr, 0, 0, &out, nullptr, nullptr),
           MSAT_EBADARG, nullptr, "env_step NULL desc");
    msat_env_desc many[MSAT_MAX_GROUPS + 1];
    for (auto &g : many) g = d;
    expect(msat_env_step_grouped(MSAT_MAX_GROUPS + 1, many, nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr,
                                 nullptr),
           MSAT_EBADARG, nullptr, "env_step_grouped too many groups");

    // network boundary (marlsat_net.h)
    expect(msat_gemm(nullptr, 4, nullptr, 4, 0, nullptr, 4, nullptr, 1, 4, 4, 0, nullptr), MSAT_EBADARG, nullptr,
           "gemm NULL");
    expect(msat_gru_ln_fused_fwd(nullptr, 0, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr, 0, nullptr, nullptr, nullptr,
                                 nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, 8, 96, nullptr),
           MSAT_EBADARG, "H must be 64, 128 or 256", "gru_ln_fused H");
    expect(msat_gru_ln_fused_fwd_h2r(nullptr, 0, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr, 0, nullptr, nullptr, nullptr,
                                     nullptr, 32, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, -1, 128,
                                     nullptr, nullptr, nullptr),
           MSAT_EBADARG, "R < 0", "gru_h2r R < 0");
    static float dummy[1024];
    int32_t idummy[4];
    expect(msat_gru_ln_bwd_g4fe(dummy, 128, dummy, 512, dummy, 128, dummy, dummy, 512, dummy + 1, 512, dummy, 128,
                                dummy, dummy + 1, nullptr, nullptr, nullptr, 0, 0, nullptr, dummy, 10, 128, 7, nullptr,
                                nullptr),
           MSAT_EBADARG, "NULL rexp", "gru_bwd_g4fe NULL rexp");
    expect(msat_gru_ln_bwd_g4f(dummy, 128, dummy, 512, dummy, 128, dummy, dummy, 512, dummy + 1, 512, dummy, 128, dummy,
                               dummy + 128, dummy, dummy, dummy, 4, 3, dummy, dummy, 10, 128, 0, nullptr),
           MSAT_EBADARG, "nfeat", "gru_bwd_g4f nfeat 3");
    expect(msat_adam(nullptr, nullptr, nullptr, nullptr, 10, 1e-3f, 0.9f, 0.999f, 1e-8f, 1, 1.0f, nullptr),
           MSAT_EBADARG, "adam", "adam NULL");
    expect(msat_adam_checked(dummy, dummy, dummy, dummy, 4, 1e-3f, 0.9f, 0.999f, 1e-8f, 0, 1.0f, idummy, nullptr),
           MSAT_EBADARG, "adam", "adam_checked count 0");
    expect(msat_set_precision(9), MSAT_EBADARG, "unknown mode 9", "set_precision 9");
    expect(msat_set_precision(MSAT_PRECISION_FP32), 0, nullptr, "set_precision fp32");
    expect(msat_get_precision(), MSAT_PRECISION_FP32, nullptr, "get_precision");
    expect(msat_gemm_wgrad_rot(dummy, 4, dummy, 4, dummy, 4, 4, 4, 4, 4, 0, dummy, nullptr), MSAT_EBADARG, "rot",
           "wgrad_rot rot == N");
    expect(msat_gemm_wgrad_h2(dummy, 4, dummy, 4, idummy, dummy, 4, 4, 4, 512, 0, 0, dummy, nullptr), MSAT_EBADARG,
           "K > 8, N <= 384", "wgrad_h2 N 512");

    // plan arithmetic: the backward's partial buffer holds the block partials and the reduction workspace
    for (int R : {1, 77, 4096, 1000000, 5000000}) {
        const size_t f = msat_gru_ln_bwd_partial_floats(R, 128);
        const size_t nb = (size_t)(R + 3) / 4 < 1024 ? (size_t)(R + 3) / 4 : 1024;
        if (f < nb * 24 * 128 + (nb + 15) / 16 * 24 * 128) {
            printf("FAIL partial_floats(%d): %zu\n", R, f);
            g_fail = 1;
        }
    }
    if (msat_gemm_wgrad_workspace_bytes(1000000, 128, 384) < 4u * 128 * 384) {
        printf("FAIL wgrad workspace\n");
        g_fail = 1;
    }
    if (msat_version() < 1) g_fail = 1;
    printf(g_fail ? "capi_host_check: FAILED\n" : "capi_host_check: ok\n");
    return g_fail;
}
