"""Run a command and report its process tree's CPU time against its wall time (are the solve
processes CPU-bound on the box's cores?).   python tools/cpu_time_of.py CMD ..."""
import os
import subprocess
import sys
import time

t0 = time.perf_counter()
rc = subprocess.run(sys.argv[1:]).returncode
wall = time.perf_counter() - t0
t = os.times()
cpu = t.children_user + t.children_system
print(f"cpu_time_of: wall {wall:.1f} s, children user {t.children_user:.1f} s + sys {t.children_system:.1f} s "
      f"= {cpu:.1f} s CPU -> {cpu / wall:.2f} cores busy on average (os.cpu_count {os.cpu_count()}, "
      f"affinity {len(os.sched_getaffinity(0))})", file=sys.stderr, flush=True)
sys.exit(rc)
