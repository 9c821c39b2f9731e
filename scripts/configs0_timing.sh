#!/bin/bash
# configs[0] on the box: the loop echo with the reference's CPU checksum
# (loop_echo_cpu) and with the GPU batches (loop_echo) -- tx coalescing on
# (the default: frames held until the work thread is idle), off
# (NET_CSUM_COALESCE=0: one fill per netif_out), and on with the resident
# queue server (NET_CSUM_QUEUE_SERVER=1) -- the same process layout, three
# runs each, plus the reference's own app/echo UDP server; and the pcap
# driver over the test double (pcap_wire), phase lines and batch sizes kept.
# Usage: scripts/configs0_timing.sh OUTDIR
set -u
out=${1:-gpurun_out/r04}
mkdir -p "$out"
B=integration/_build
: > "$out/configs0_timing.txt"
keep="^timing|echoed intact|^engine|^batch sizes"
run() { # label env... exe args...
  # rc 1 = the echo's own check failed (the reference's TCP occasionally hands
  # back a segment's header in place of its data, CPU build too: DESIGN.md §2);
  # the run's lines are kept and the next one starts.  Anything else (a
  # crash, a time-out) ends the script.
  local label=$1; shift
  echo "== $label" >> "$out/configs0_timing.txt"
  timeout -k 10 120 env "$@" > "$out/run.raw" 2>&1
  local rc=$?
  grep -E "$keep|^tcp: echoed bytes differ|^tcp: (got|sent) " "$out/run.raw" >> "$out/configs0_timing.txt"
  if [ $rc -eq 1 ]; then echo "   (rc 1: echo check failed)" >> "$out/configs0_timing.txt"; return 0; fi
  [ $rc -eq 0 ] || { echo "$label failed rc=$rc"; tail -20 "$out/run.raw"; exit $rc; }
}
for rep in 1 2 3; do
  run "loop_echo_cpu rep $rep" X=0 $B/loop_echo_cpu --rounds 2000 --tcp-bytes 1048576
  run "loop_echo_cpu rep $rep, reference udp_echo_server" X=0 $B/loop_echo_cpu --ref-udp-server --udp-only --rounds 2000
  run "loop_echo coalesce rep $rep" X=0 $B/loop_echo --rounds 2000 --tcp-bytes 1048576
  run "loop_echo coalesce rep $rep, reference udp_echo_server" X=0 $B/loop_echo --ref-udp-server --udp-only --rounds 2000
  run "loop_echo no-coalesce rep $rep" NET_CSUM_COALESCE=0 $B/loop_echo --rounds 2000 --tcp-bytes 1048576
  run "loop_echo coalesce+queue-server rep $rep" NET_CSUM_QUEUE_SERVER=1 $B/loop_echo --rounds 2000 --tcp-bytes 1048576
done
rm -f "$out"/run.raw
timeout -k 10 200 $B/pcap_wire tests/golden > "$out/pcap_wire.raw" 2>&1
rc=$?
grep -o "phase [a-z_]*: .*\|pcap netif.*\|^engine.*\|^batch sizes.*\|pcap_wire: .*" "$out/pcap_wire.raw" > "$out/pcap_wire_gpu.txt"
rm -f "$out/pcap_wire.raw"
exit $rc
