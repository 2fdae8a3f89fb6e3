"""Load the golden fixtures written by tools/gen_golden.py (data only)."""
import glob
import json
import os
from collections import OrderedDict

import numpy as np

from oracle import BF16

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _arr(z, name, dtypes):
    a = z[name]
    if dtypes.get(name) == 'bfloat16':
        return BF16(a)
    if dtypes.get(name) == 'b64':          # gRPC upload text
        return a.tobytes().decode('ascii')
    return a


def load_case(name):
    path = os.path.join(GOLDEN, name + '.npz')
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z['meta']))
        dts = meta['dtypes']
        clients = []
        for i in range(meta['n']):
            d = OrderedDict()
            for k in meta['keys'][i]:
                d[k] = _arr(z, 'x|%d|%s' % (i, k), dts)
            clients.append((meta['sizes'][i], d))
        out = OrderedDict((k, _arr(z, 'out|' + k, dts))
                          for k in meta['out_keys'])
        init = None
        if 'init_keys' in meta:
            init = OrderedDict((k, _arr(z, 'init|' + k, dts))
                               for k in meta['init_keys'])
        extra = {n[len('extra|'):]: z[n] for n in z.files
                 if n.startswith('extra|')}
    return meta, clients, out, init, extra


def case_names(prefix=''):
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(GOLDEN, prefix + '*.npz')))
