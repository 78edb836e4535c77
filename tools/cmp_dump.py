"""Compare two tools/dump_kernels.py outputs bit for bit: python tools/cmp_dump.py a.npz b.npz"""
import sys, numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = [k for k in a.files if k not in b.files or a[k].shape != b[k].shape or not np.array_equal(a[k], b[k])]
print(len(a.files), "arrays;", "identical" if not bad else f"DIFFER: {bad}")
