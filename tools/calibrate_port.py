"""Speed calibration of the CPU restatement (oracle/, the bench's `cpu_baseline` "port") against the
reference itself, on the same cores of the build container (record t_port / t_ref).

    python tools/calibrate_port.py [--cores 6,7] [--repeats 2] [key ...]

Each key (e.g. maxcut_10_r1_s41) runs as two single-thread processes at once, the reference
(tests/golden/make_golden.py `one`, PYTHONHASHSEED=0) on one core and the port (bench._cpu_worker,
full solve) on the other, then again with the cores swapped.  Both time the IPM loop only
(reference: src/utils.py:272-302's (t3 - t2) / num_iters; port: the same span).  Prints one JSON line
per key; build-container only (the reference is not on the GPU box)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PROBLEM = {"maxcut": "maxcut", "corr": "corr_clust", "graphm": "graphm"}

PORT = r"""
import sys, io, contextlib
sys.path.insert(0, {root!r})
import bench
sys.stdin = io.StringIO("go\n")
bench._cpu_worker({problem!r}, {cfg!r}, {seed}, {rank}, 0)
"""


def parse(key):
    cfg, r, s = key.rsplit("_", 2)
    return cfg, int(r[1:]), int(s[1:])


def launch(kind, key, core, tmp):
    cfg, rank, seed = parse(key)
    prob = PROBLEM[cfg.split("_")[0]]
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", PYTHONHASHSEED="0")
    if kind == "ref":
        cmd = [sys.executable, os.path.join(ROOT, "tests", "golden", "make_golden.py"), "one", prob, cfg, str(seed),
               str(rank), "0", tmp, "0"]
        return subprocess.Popen(["taskset", "-c", str(core)] + cmd, env=env, stdout=subprocess.DEVNULL, cwd=ROOT)
    code = PORT.format(root=ROOT, problem=prob, cfg=os.path.join(ROOT, "configs", cfg + ".yaml"), seed=seed,
                       rank=rank)
    return subprocess.Popen(["taskset", "-c", str(core), sys.executable, "-c", code], env=env,
                            stdout=open(tmp, "w"), stderr=subprocess.DEVNULL, cwd=ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cores", default="6,7")
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("keys", nargs="*")
    a = ap.parse_args()
    cores = [int(c) for c in a.cores.split(",")]
    keys = a.keys or ["maxcut_5_r1_s0", "maxcut_10_r1_s41", "maxcut_10_r1_s235", "maxcut_10_r1_s35",
                      "maxcut_10_r1_s14"]
    for key in keys:
        ref, port = [], []
        for rep in range(a.repeats):
            c_ref, c_port = (cores[0], cores[1]) if rep % 2 == 0 else (cores[1], cores[0])
            with tempfile.TemporaryDirectory() as d:
                tr, tp = os.path.join(d, "ref.json"), os.path.join(d, "port.json")
                pr, pp = launch("ref", key, c_ref, tr), launch("port", key, c_port, tp)
                if pr.wait() != 0 or pp.wait() != 0:
                    print(json.dumps({"key": key, "error": [pr.returncode, pp.returncode]}), flush=True)
                    break
                R = json.load(open(tr))
                P = json.loads(open(tp).read().strip().splitlines()[-1])
                ref.append([R["num_iters"], R["sec_per_iter"]])
                port.append([P["full_solve_iters"], P["full_solve_s_per_iter"]])
        if not ref or len(ref) != len(port):
            continue
        r = min(x[1] for x in ref)
        p = min(x[1] for x in port)
        print(json.dumps({"key": key, "ref": ref, "port": port, "ref_s_per_iter": r, "port_s_per_iter": p,
                          "port_over_ref": p / r}), flush=True)


if __name__ == "__main__":
    main()
