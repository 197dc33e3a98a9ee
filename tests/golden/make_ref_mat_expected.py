"""Expected contents of the two MATLAB-written MAT files the reference holds
(Simulation/FIR.mat, Simulation/file.mat; copied byte-for-byte into tests/golden/ref_mat/
as data fixtures).  Decoded with scipy.io.loadmat (a data-only loader) into
ref_mat/expected.json, which tests/test_matio.py compares librsp's native reader with.
Run from the repo root: python tests/golden/make_ref_mat_expected.py
"""
import json
import os

import scipy.io as sio

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ref_mat')
out = {}
for fn in ('FIR.mat', 'file.mat'):
    d = sio.loadmat(os.path.join(HERE, fn))
    ent = {}
    for k, v in d.items():
        if k.startswith('__'):
            continue
        if v.dtype.kind == 'U':
            ent[k] = {'class': 'char', 'value': str(v[0])}
        else:
            ent[k] = {'class': 'double', 'size': list(v.shape), 'value': v.ravel(order='F').tolist()}
    out[fn] = ent
json.dump(out, open(os.path.join(HERE, 'expected.json'), 'w'), indent=1, ensure_ascii=False)
print(json.dumps(out, ensure_ascii=False)[:300])
