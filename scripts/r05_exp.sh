#!/bin/bash
# round 5 experiments (one box): last-error before/after, descriptor
# prefetch distance, the packed fallback, the mixed line's order
set -u
out=gpurun_out/r05b
mkdir -p $out
scripts/gpu_steps.sh \
  "lasterr_ab:120:python -u scripts/lasterror_ab.py abl/libtcsum_r04.so tcp_amd/libtcsum.so > $out/lasterror_ab.txt" \
  "pk_layouts:420:python -u scripts/pk_layouts_ab.py mtu,shuffled,ragged,small packed=0 lib=abl/libtcsum_r04.so pf_dist=1024 pf_dist=2048 pf_dist=4096 > $out/pk_layouts_pf.txt" \
  "mixed_pf:300:python -u scripts/env_ab.py mixed pf_dist=1024 pf_dist=2048 pf_dist=4096 > $out/mixed_pf.txt" \
  "rx_pf:300:python -u scripts/env_ab.py mixed_rx pf_dist=2048 pf_dist=4096 > $out/mixed_rx_pf.txt" \
  "ipv4_db:400:python -u scripts/ipv4_shape_ab.py mixed mixed_rx --db > $out/ipv4_db.txt" \
  "tso_pf:300:python -u scripts/env_ab.py tso pf_dist=512 pf_dist=1024 pf_dist=2048 > $out/tso_pf.txt" \
  "ipv4_r04:300:python -u scripts/ab_lib.py tcp_amd/libtcsum.so abl/libtcsum_r04.so mixed,mixed_rx,mixed_tx > $out/ab_r04_ipv4.txt" \
  "calib:300:python -u scripts/pmc_calib.py $out/pmc_calib.json > $out/pmc_calib.txt"
