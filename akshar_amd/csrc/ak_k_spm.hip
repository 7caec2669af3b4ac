// ak_k_spm.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

int launch_spm(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 0: return launch_rows<OP_SPM, 0>(w, a, out_offs, st);
        case 1: return launch_rows<OP_SPM, 1>(w, a, out_offs, st);
        case 2: return launch_rows<OP_SPM, 2>(w, a, out_offs, st);
        case 3: return launch_rows<OP_SPM, 3>(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "spm: unsupported flags");
}

}  // namespace ak
