"""Time acmi_kfac_inverse (all 12 damped fp64 inverses of the ACKTR factors) on
random SPD factors of the bench's shapes."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'actor-critic_amd'))
from actorcritic import _lib  # noqa: E402


def main(iters=10):
    lib = _lib.load()
    A, C3 = 4, 32
    din, dout, so = (ctypes.c_int64 * 6)(), (ctypes.c_int64 * 6)(), (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    rng = np.random.default_rng(5)
    fac = np.zeros(tot.value, np.float32)
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        x = rng.standard_normal((n + 3, n)).astype(np.float32)
        fac[so[f]:so[f] + n * n] = (x.T @ x / x.shape[0]).ravel()
    dev = torch.device('cuda:0')
    fac_d = torch.from_numpy(fac).to(dev)
    inv = torch.zeros(lib.acmi_kfac_inverse_floats(A, C3), device=dev)
    ws = torch.zeros(lib.acmi_kfac_inverse_ws_doubles(A, C3), dtype=torch.float64, device=dev)

    def run():
        _lib.call('acmi_kfac_inverse', A, C3, _lib.ptr(fac_d), ctypes.c_float(0.01), 0, _lib.ptr(inv),
                  _lib.ptr(ws), _lib.stream_handle())

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({'ms_per_inverse': e0.elapsed_time(e1) / iters, 'checksum': float(inv.double().sum()),
                      'sha': hashlib.sha1(inv.cpu().numpy().tobytes()).hexdigest()[:16]}))


if __name__ == '__main__':
    main()
