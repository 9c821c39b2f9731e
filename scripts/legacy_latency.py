"""Per-call latency of the synchronous drop-in symbols: blocking stream sync
vs polling a completion word the stream writes (the default; TCSUM_SYNC=block
forces the blocking sync)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = """
import sys, json; sys.path.insert(0, %r)
import bench, tcp_amd
print(json.dumps(bench.legacy_latency(tcp_amd)))
""" % ROOT
for mode in ("block", "poll", "block", "poll"):  # "poll": anything but "block"
    env = dict(os.environ, TCSUM_SYNC=mode)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print(mode, r.stdout.strip() or r.stderr[-500:])
