"""Compare two tools/dump_kernels.py outputs bit for bit: python tools/npz_equal.py a.npz b.npz"""
import numpy as np, sys
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("cases", len(a.files), "bit-identical" if not bad else f"DIFFER: {bad[:10]}")
