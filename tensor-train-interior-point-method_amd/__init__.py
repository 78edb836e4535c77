"""ttipm_amd -- MI355X-native TT-IPM Newton/KKT hot path (package dir:
`tensor-train-interior-point-method_amd/`, import alias `ttipm_amd`, see ../ttipm_amd.py).

Host code mirrors the reference's interface (`src/tt_ops.py`, `src/tt_als.py`, `src/tt_ipm.py`,
`psd_system/*/create_problem`, `src/utils.py::run_experiment`); TT cores are fp64 tensors on the
GPU and every arithmetic op runs in hand-written HIP kernels behind the C ABI `include/ttk.h`
(`libttk.so`).  There is no CPU fallback: importing the numeric modules without the built
library raises."""
