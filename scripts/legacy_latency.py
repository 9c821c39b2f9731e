"""Per-call latency of the synchronous drop-in symbols: blocking stream sync
vs polling a completion word the stream writes (the default; debug knob
sync_block=1 forces the blocking sync)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = """
import sys, json; sys.path.insert(0, %r)
import bench, tcp_amd
tcp_amd.debug_set("sync_block", int(sys.argv[1])); tcp_amd.debug_set("args_launch", int(sys.argv[2]))
print(json.dumps(bench.legacy_latency(tcp_amd)))
""" % ROOT
runs = [("block", "1"), ("poll", "0"), ("poll", "1")] * 2  # (sync_block, args_launch)
for mode, inl in runs:  # args_launch=0: descriptor (and bytes) via pinned memory
    r = subprocess.run([sys.executable, "-c", code, "1" if mode == "block" else "0", inl], capture_output=True,
                       text=True)
    print(mode, "args" if inl == "1" else "pinned-desc", r.stdout.strip() or r.stderr[-500:])
