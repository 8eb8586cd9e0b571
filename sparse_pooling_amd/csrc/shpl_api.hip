// shpl_api.hip -- version / status strings of the libshpl C ABI.
#include "shpl_common.h"

extern "C" const char *shpl_version(void) { return "shpl 0.1.0 (gfx950)"; }

extern "C" const char *shpl_status_string(int status) {
    switch (status) {
        case SHPL_OK: return "ok";
        case SHPL_ERR_BAD_SHAPE: return "inconsistent shape, stride or alignment";
        case SHPL_ERR_INDEX_OOB: return "index out of bounds";
        case SHPL_ERR_HIP: return "HIP runtime error";
        case SHPL_ERR_WORKSPACE: return "workspace too small";
        case SHPL_ERR_ARG: return "invalid argument";
        default: return "unknown status";
    }
}
