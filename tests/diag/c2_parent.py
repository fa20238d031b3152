"""C2 (bin/speed_replica) run from a Python parent in three states, alternating: nothing loaded;
libsiftgpu imported (as bench.py's module imports do); HIP runtime initialised (device count).
  python tests/diag/c2_parent.py  (GPU box)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from sift_synth import synth_image  # noqa: E402

pgm = "/tmp/c2p.pgm"
img = synth_image(1920, 1080, 2000)
open(pgm, "wb").write(b"P5\n1920 1080\n255\n" + img.tobytes())
exe = os.path.join(ROOT, "modify-sift-gpu_amd", "bin", "speed_replica")


def run(tag):
    r = subprocess.run([exe, "30", "--", "-i", pgm, "-fo", "0", "-no", "4", "-d", "3"],
                       capture_output=True, text=True, timeout=120)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    print(tag, d["avg_ms"], flush=True)


for i in range(3):
    run("plain")
import sgpu  # noqa: E402
for i in range(3):
    run("imported")
sgpu.lib()
for i in range(3):
    run("lib()")
sgpu.device_count()
for i in range(3):
    run("device_count")
