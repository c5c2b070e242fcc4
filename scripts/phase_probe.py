"""Time the sorted count with the bucket kernel stopped after each phase."""
import json, os, subprocess, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for ph in ["0", "1", "2", "99"]:
    env = dict(os.environ, FASTKMER_DEBUG_PHASE=ph)
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "count_once.py")], env=env,
                         capture_output=True, text=True)
    print("phase", ph, out.stdout.strip(), out.stderr.strip()[-300:], flush=True)
