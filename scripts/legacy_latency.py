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
runs = [("block", "1"), ("poll", "0"), ("poll", "1")] * 2  # (TCSUM_SYNC, TCSUM_INLINE)
for mode, inl in runs:  # "poll": anything but "block"; TCSUM_INLINE=0: checksum16 bytes staged, not in the kernel arguments
    env = dict(os.environ, TCSUM_SYNC=mode, TCSUM_INLINE=inl)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print(mode, "inline" if inl == "1" else "staged", r.stdout.strip() or r.stderr[-500:])
