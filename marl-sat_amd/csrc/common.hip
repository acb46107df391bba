// Error channel of the C-ABI: a thread-local message + negative return codes.
#include "common.h"

namespace msat {

static thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch_plain(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MSAT_EHIP, "%s: %s", what, hipGetErrorString(e));
    return MSAT_OK;
}

}  // namespace msat

extern "C" const char *msat_last_error(void) { return msat::g_err; }
// ABI version: 2 since msat_step_out gained clock_stamps (round 5), 3 since msat_env_state gained reset_queue /
// reset_serial (round 6); a caller built against an older header passes structs without those fields, so it must
// check msat_version() >= 3
extern "C" int msat_version(void) { return 3; }
