// ak_k_bpe_f01.hip — one-lane-per-row BPE for clean_hinglish=False (flags 0 / 1): normalize_text
// is NFC (+ Roman lowercasing), any text reaches the tokenizer, so the row sink is BpeSink<true>:
// the added-token split, HF's full NFKC (Unicode 9 NFKD, HF ccc, HF composites) and the
// Whitespace pre-tokenizer over every code point (ak_dev.h). Staged slots: a row's ids never
// exceed 6 x its bytes + 2 (U+FDFA, 3 bytes, is 18 code points after NFKD; tools/gen_tables.py).
#include "ak_internal.h"

namespace ak {

constexpr uint32_t BPE_NFKC_MUL = 6;

int launch_bpe_f01(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    if (flags == 1) return launch_rows_staged<OP_BPE, 1>(w, a, out_offs, st, BPE_NFKC_MUL, BPE_ADD);
    return launch_rows_staged<OP_BPE, 0>(w, a, out_offs, st, BPE_NFKC_MUL, BPE_ADD);
}

}  // namespace ak
