"""A/B of two libofx builds on the gn_2k fixture chain: prints one JSON line of output digests, so two runs with
OFX_LIB pointing at different builds show whether a change kept the solve bit for bit.

    OFX_LIB=tools/ablib/libofx_prev.so python tools/ab_gn.py ; python tools/ab_gn.py
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tests.test_gpu_golden_gn import _load, _chain  # noqa: E402


def main():
    cuda = torch.device("cuda:0")
    out = {"lib": os.environ.get("OFX_LIB", "libofx.so")}
    for name in ("gn_2k.npz", "gn_4k.npz"):
        g = _load(name)
        s, outs = _chain(g, cuda, prefetch=True)
        h = hashlib.sha256()
        for o in outs:
            h.update(o["node_rotations"].cpu().numpy().tobytes())
            h.update(o["node_translations"].cpu().numpy().tobytes())
            h.update(np.asarray(o["convergence_info"]["total"], dtype=np.float64).tobytes())
        out[name] = {"digest": h.hexdigest()[:16],
                     "pcg_iters": [int(o["convergence_info"]["pcg_iterations"]) for o in outs]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
