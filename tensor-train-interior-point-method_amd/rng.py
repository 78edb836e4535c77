"""The NumPy random stream of the solve path, per host thread.

The reference draws its random TT cores, kick vectors and core indices from NumPy's global legacy
MT19937 (`np.random.randn / randint`, seeded in `src/utils.py:258-262`).  A thread that runs a
solve while other threads in the same process run theirs (bench.py's solves in flight) gets a
private `RandomState` here; every other thread draws from NumPy's global one, so single-solve use
is exactly the reference's stream.  A RandomState given the global stream's state produces the
same draws as the global functions."""
import threading

import numpy as np

_TL = threading.local()


def R():
    """This thread's RandomState: a private one after `private()`, else NumPy's global one."""
    rs = getattr(_TL, "rs", None)
    return rs if rs is not None else np.random.mtrand._rand


def private():
    """Give the calling thread its own MT19937 stream (state set by the solve it runs)."""
    _TL.rs = np.random.RandomState()
    return _TL.rs
