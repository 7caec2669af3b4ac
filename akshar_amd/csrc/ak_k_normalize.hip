// ak_k_normalize.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

int launch_normalize(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 0: return launch_rows<OP_NORMALIZE, 0>(w, a, out_offs, st);
        case 1: return launch_rows<OP_NORMALIZE, 1>(w, a, out_offs, st);
        case 2: return launch_rows<OP_NORMALIZE, 2>(w, a, out_offs, st);
        case 3: return launch_rows<OP_NORMALIZE, 3>(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "normalize: unsupported flags");
}

}  // namespace ak
