#!/bin/bash
# configs[0] on the box: the loop echo with the reference's CPU checksum
# (loop_echo_cpu) and with the GPU batches (loop_echo), the same process
# layout, three runs each, plus the reference's own app/echo UDP server; and
# the pcap driver over the test double (pcap_wire), phase lines kept.
# Usage: scripts/configs0_timing.sh OUTDIR
set -u
out=${1:-gpurun_out/r03}
mkdir -p "$out"
B=integration/_build
: > "$out/configs0_timing.txt"
for rep in 1 2 3; do
  for exe in loop_echo_cpu loop_echo; do
    echo "== $exe rep $rep (--rounds 2000 --tcp-bytes 1048576)" >> "$out/configs0_timing.txt"
    timeout -k 10 120 $B/$exe --rounds 2000 --tcp-bytes 1048576 > "$out/$exe.raw" 2>&1 || { echo "$exe failed rc=$?"; tail -20 "$out/$exe.raw"; exit 1; }
    grep -E "^timing|echoed intact|^engine" "$out/$exe.raw" >> "$out/configs0_timing.txt"
    echo "== $exe rep $rep, reference app/echo/udp_echo_server.c (--ref-udp-server --udp-only --rounds 2000)" >> "$out/configs0_timing.txt"
    timeout -k 10 120 $B/$exe --ref-udp-server --udp-only --rounds 2000 > "$out/$exe.raw" 2>&1 || { echo "$exe ref failed rc=$?"; tail -20 "$out/$exe.raw"; exit 1; }
    grep -E "^timing|echoed intact|^engine" "$out/$exe.raw" >> "$out/configs0_timing.txt"
  done
done
rm -f "$out"/*.raw
timeout -k 10 200 $B/pcap_wire tests/golden > "$out/pcap_wire.raw" 2>&1
rc=$?
grep -o "phase [a-z_]*: .*\|pcap netif.*\|^engine.*\|pcap_wire: .*" "$out/pcap_wire.raw" > "$out/pcap_wire_gpu.txt"
rm -f "$out/pcap_wire.raw"
exit $rc
