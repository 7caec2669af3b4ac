import sys, gzip, json, os
sys.path.insert(0, '.')
import numpy as np
from akshar_amd import engine
from tests.util import rows_ints
gold = [json.loads(l) for l in gzip.open('tests/golden/golden.jsonl.gz', 'rt')]
rows = [r for r in gold if r['set'] != 'long']
m = engine.SPM('models/akshar.model')
buf, offs = engine.pack([r['text'] for r in rows])
for path in (1, 0):
    ids, oo = m.encode_batch(buf, offs, path=path)
    got = rows_ints(ids.cpu().numpy(), oo.cpu().numpy())
    bad = [(r['set'], r['i']) for r, g in zip(rows, got) if g != r['spm']]
    print(os.environ.get('AK_LIB_VARIANT', 'default'), 'path', path, 'bad', len(bad), bad[:4], flush=True)
# single rows
for t in ['मैं स्कूल जा रहा हूँ', 'स्कूल', 'कू']:
    b, o = engine.pack([t])
    ids, oo = m.encode_batch(b, o)
    print(t, ids.cpu().tolist(), flush=True)
