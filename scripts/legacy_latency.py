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
runs = [("block", "1"), ("poll", "0"), ("poll", "1")] * 2  # (TCSUM_SYNC, TCSUM_ARGS_LAUNCH)
for mode, inl in runs:  # "poll": anything but "block"; TCSUM_ARGS_LAUNCH=0: descriptor (and bytes) via pinned memory
    env = dict(os.environ, TCSUM_SYNC=mode, TCSUM_ARGS_LAUNCH=inl)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print(mode, "args" if inl == "1" else "pinned-desc", r.stdout.strip() or r.stderr[-500:])
