"""CP iteration time graph-replayed vs eager (RAOCP_EAGER) at a config: python tools/graph_check.py <cfg> [dtype]"""
import os
import subprocess
import sys

cfg = sys.argv[1]
dt = sys.argv[2] if len(sys.argv) > 2 else ("float32" if cfg == "5" else "float64")
for eager in ("0", "1"):
    for K in ("24", "48", "96"):
        env = dict(os.environ, RAOCP_EAGER=eager)
        out = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "prof_cp.py"), cfg, K, dt], env=env,
                             capture_output=True, text=True, timeout=200)
        print(f"eager={eager} K={K}: {out.stdout.strip()} {out.stderr.strip()[-300:]}", flush=True)
