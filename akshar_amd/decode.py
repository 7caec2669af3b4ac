"""id -> token-string maps for tokenize() with a model (tokenizer.py:152-156: enc.tokens /
EncodeAsPieces). Decoding ids to text runs on the device (ak_bpe_decode / ak_spm_decode,
akshar_amd/csrc/ak_k_decode.hip; engine.decode_lists)."""
def bpe_tokens(model, ids):
    return [model.id_to_token[i] for i in ids]


def spm_pieces(model, ids):
    return [model.pieces[i].decode("utf-8", "surrogatepass") for i in ids]
