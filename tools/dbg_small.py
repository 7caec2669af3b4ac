import sys, os
sys.path.insert(0, "/root/repo")
from akshar_amd.tokenizer import aksharTokenizer
bpe = aksharTokenizer(model_path="/root/repo/models/akshar.json", model_type="bpe")
texts = ["aaj mausam", "hello world", "क्षेत्रे", "x", "", "Heyyy यार kya HAAL hai"]
batch = bpe.encode_batch(texts + ["z"])[:-1]
for t, b in zip(texts, batch):
    one = bpe.encode(t)
    print(repr(t), "one", one, "batch", b, "OK" if one == b else "BAD")
for t, b in zip(texts, batch):
    one = bpe.encode(t)
    print(repr(t), "again", one, "OK" if one == b else "BAD")
