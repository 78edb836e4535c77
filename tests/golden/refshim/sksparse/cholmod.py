"""Golden-vector generation shim: scikit-sparse is imported by src/tt_als.py:10 but SpCholInv is dead code."""


def cholesky(*a, **k):
    raise RuntimeError("scikit-sparse is not available in this image")
