// ak_k_bpe.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

int launch_bpe(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 2: return launch_rows<OP_BPE, 2>(w, a, out_offs, st);
        case 3: return launch_rows<OP_BPE, 3>(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "bpe: unsupported flags");
}

}  // namespace ak
