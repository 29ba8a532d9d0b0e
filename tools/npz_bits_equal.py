"""Compare two .npz files array by array, bit for bit (NaN payloads included),
except keys matching an optional substring list given after --float-close
(compared with numpy.allclose, rtol 1e-12): python tools/npz_bits_equal.py A B."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
close = sys.argv[sys.argv.index("--float-close") + 1:] if "--float-close" in sys.argv else []
bad = []
for k in sorted(a.files):
    x, y = a[k], b[k]
    if any(c in k for c in close):
        ok = np.allclose(x, y, rtol=1e-12, atol=0, equal_nan=True)
    else:
        ok = x.shape == y.shape and x.tobytes() == y.tobytes()
    print(f"{k}: {'same' if ok else 'DIFFERENT'}")
    if not ok:
        bad.append(k)
sys.exit(1 if bad else 0)
