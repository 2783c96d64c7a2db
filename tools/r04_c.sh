#!/bin/bash
# race study, second pass: details of the differing entries, no-T-stash, and fe/fx roles
set -o pipefail
R=$PWD
for v in 1; do
  for env in "PROBE_DETAIL=1" "PROBE_DETAIL=1 PROBE_NO_T=1" "PROBE_DETAIL=1 PROBE_SWAP=1"; do
    echo "== race$v $env"
    env $env MPVAE_HIP_LIB="$R/abl/race$v/libmpvae_hip.so" timeout -k 10 120 \
      python tools/repeat_probe.py 512 2000 128 128 40 || exit $?
  done
done
