import sys
sys.path.insert(0, '.')
from akshar_amd import engine
m = engine.SPM('models/akshar.model')
b, o = engine.pack(['स्कूल'])
ids, oo = m.encode_batch(b, o)
import torch; torch.cuda.synchronize()
print('ids', ids.cpu().tolist(), flush=True)
