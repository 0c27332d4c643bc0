#!/bin/bash
# Interleaved A/B of transform variants against the default library and an alternative build
# (AB_LIB2 = library file name under alpenglow_amd/_lib); every GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/ab_xform.py ${AB_ARGS:-} > gpurun_out/ab_a$i.json 2> gpurun_out/ab_a$i.err
  rc=$?; echo "lib1 run $i exit $rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  AG_RS_LIB_NAME=${AB_LIB2} timeout -k 10 200 python tools/ab_xform.py ${AB_ARGS2:-$AB_ARGS} > gpurun_out/ab_b$i.json 2> gpurun_out/ab_b$i.err
  rc=$?; echo "lib2 run $i exit $rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
python - <<'PY'
import json
for n in ("a1","b1","a2","b2"):
    d=json.load(open(f"gpurun_out/ab_{n}.json"))
    print(n, {v:(round(r["enc_ms"],4), round(r["dec_ms"],4)) for v,r in d.items()})
PY
