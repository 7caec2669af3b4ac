// ak_k_bpe_f2.hip — one-lane-per-row BPE (staged row kernel + slow / huge tiers) for flags 2
// (normalize_roman=False), and the flags dispatcher of the BPE row path (flags 0 / 1:
// ak_k_bpe_f01.hip, flags 3: ak_k_bpe_f3.hip).
#include "ak_internal.h"

namespace ak {

int launch_bpe_f3(AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_bpe_f01(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);

int launch_bpe(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 0:
        case 1: return launch_bpe_f01(flags, w, a, out_offs, st);
        case 2: return launch_rows_staged<OP_BPE, 2>(w, a, out_offs, st, BPE_MUL, BPE_ADD);
        case 3: return launch_bpe_f3(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "bpe: unsupported flags");
}

}  // namespace ak
