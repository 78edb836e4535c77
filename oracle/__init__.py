"""oracle/ -- CPU restatement of the reference TT-IPM hot path.  TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / CPU baseline -- never as the thing measured or shipped.
The MI355X product (`tensor-train-interior-point-method_amd/`, imported as `ttipm_amd`) does not
import it and fails loudly if its HIP library is missing.

Pinning: the restatement is checked against golden vectors produced by the reference itself
(`tests/golden/make_golden.py`: the reference's own Python + its Cython kernels compiled from
source by `oracle/build_ref.py`), with two third-party packages absent from the image replaced
in that script only: opt_einsum (contraction-order planner -> numpy.einsum greedy, same sums)
and petsc4py's KSPLGMRES (-> `oracle/petsc_lgmres.py`, a restatement of PETSc's published
algorithm; parity against real PETSc is UNPINNED, see that module).

Modules: `tt` (TT algebra, `cy_src/tt_ops_cy.pyx` + `src/tt_ops.py`), `als` (block TT + AMEn,
`src/tt_als.py:12-825,1502-1768`), `eig` (step-size ALS, `src/tt_als.py:876-1499`),
`ipm` (local KKT solvers + IPM loop, `src/tt_ipm.py`), `problems` (generators + runner record),
`petsc_lgmres`."""
