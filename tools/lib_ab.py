"""Same-box A/B of two prebuilt libraries (FLC_LIB): tools/env_ab.py's workloads (the headline step, the encode alone,
f1, configs[2]'s 25 M top-k step, a 25 M stacked encode), run as separate processes, interleaved A B A B A B.
    python tools/lib_ab.py ab/libflc_A.so ab/libflc_B.so [more .so ...] [rounds]"""
import os
import subprocess
import sys

libs = [a for a in sys.argv[1:] if a.endswith(".so")]
rest = [a for a in sys.argv[1:] if not a.endswith(".so")]
rounds = int(rest[0]) if rest else 3
here = os.path.dirname(os.path.abspath(__file__))
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, FLC_LIB=lib, FLC_AB_LABEL=os.path.basename(lib))
        out = subprocess.run([sys.executable, os.path.join(here, "env_ab.py"), "FLC_AB_LABEL"], env=env,
                             capture_output=True, text=True, timeout=180)
        if out.returncode != 0:
            print(out.stderr[-2000:], flush=True)
            sys.exit(1)
        print([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1], flush=True)
