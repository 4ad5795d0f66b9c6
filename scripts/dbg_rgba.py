import sys, os
sys.path.insert(0, 'go-webp_amd'); sys.path.insert(0, 'tests')
import numpy as np, webp_amd
from oracle_lib import load_lossy, lossy_cases
names = [n for n in lossy_cases() if n != 'alpha_64x48']
ctx = webp_amd.Context(0)
for single in (True, False):
    datas = [load_lossy(n)[0] for n in names]
    golds = [load_lossy(n)[1] for n in names]
    if single:
        for n, d, g in zip(names, datas, golds):
            b = ctx.batch([d]); b.run(); r = b.rgba(0); b.close()
            bad = np.argwhere((r != g['rgba']).any(-1))
            print('single', n, r.shape, len(bad), bad[:8].tolist())
    else:
        b = ctx.batch(datas); b.run()
        for i, (n, g) in enumerate(zip(names, golds)):
            r = b.rgba(i)
            bad = np.argwhere((r != g['rgba']).any(-1))
            print('batch', n, len(bad), bad[:8].tolist(), r[tuple(bad[0])].tolist() if len(bad) else '', g['rgba'][tuple(bad[0])].tolist() if len(bad) else '')
        b.close()
ctx.close()
