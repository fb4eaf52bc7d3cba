"""Digest of one fixed backward (grads + A factors + G factors) at M images, for
bit-identity A/Bs of library builds (ACMI_LIB=... python scripts/bwd_digest.py)."""
import ctypes
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))
import torch  # noqa: E402

from actorcritic import _lib  # noqa: E402


def main(M):
    from actorcritic._engine import NetEngine
    eng = NetEngine(4, 32)
    g = torch.Generator(device='cuda').manual_seed(5)
    obs = torch.randint(0, 256, (M, 84, 84, 4), dtype=torch.uint8, device='cuda', generator=g)
    acts = eng.activations(M)
    eng.forward(obs.data_ptr(), M, acts.struct)
    st = eng.update_state(M)
    st.dhead.normal_(generator=g)
    st.dhead[:, 5:] = 0

    class F:
        pass
    f = F()
    f.obs, f.M, f.acts = obs, M, acts
    eng.backward(f, st, True)
    eng.output_stats(f, st, 7, 3)
    torch.cuda.synchronize()
    for name, t in (('grads', st.grads), ('astat', st.astat), ('gstat', st.gstat)):
        print(name, hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16])


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10240)
