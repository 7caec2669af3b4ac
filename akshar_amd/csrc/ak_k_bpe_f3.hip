// ak_k_bpe_f3.hip — one-lane-per-row BPE (staged row kernel + slow / huge tiers) for flags 3
// (normalize_text defaults): the reference path for rows the tile kernel does not take, and
// ak_ws_set_tiling(ws, 0, ...). Each (op, flags) instantiation is its own TU so hipcc builds them in
// parallel.
#include "ak_internal.h"

namespace ak {

int launch_bpe_f3(AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    return launch_rows_staged<OP_BPE, 3>(w, a, out_offs, st, BPE_MUL, BPE_ADD);
}

}  // namespace ak
