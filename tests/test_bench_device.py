"""bench.py's own device branches run as a fresh child process on the GPU (the driver's
form): BASELINE configs[4]'s `strong_stream` sub-line and the host-memory (`--pcie`) leg
with its NUMA placement, both verified on the device by the bench itself.

Reference: independent slices, /root/reference/src/shredder/reed_solomon.rs:88-231; the
host-memory arrival of blocks, disseminator/rotor.rs:108-112, network/udp.rs:9-12."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_strong_stream_and_pcie_on_device():
    """`--strong-stream 4096` at N = 1 times the same 4096 x 1 MiB workload as the weak line
    as a configs[4]-style stream (block g seeded by its global index): it must verify on the
    device, start at block 0, and run within 10 % of the weak line's rate.  `--pcie` moves
    256 blocks through pinned host staging bound to the GPU's NUMA node and must reproduce
    the device result."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "10",
                        "--warmup", "2", "--no-cpu-baseline", "--strong-stream", "4096", "--pcie",
                        "--pcie-blocks", "256"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["verify"]["all_ranks_ok"] is True and line["verify"]["reconstruct_restores_all_blocks"]
    sub = line["strong_stream"]
    assert sub["verify"] == {"per_rank": [True], "all_ranks_ok": True}
    assert sub["first_block"] == [0] and sub["blocks_per_rank"] == [4096] and sub["stream_blocks"] == 4096
    assert abs(sub["value"] / line["value"] - 1) < 0.10, (sub["value"], line["value"])
    pc = line["pcie_inclusive"]
    assert pc["matches_device_result"] is True and pc["blocks"] == 256
    assert pc["numa"]["bdf"] and isinstance(pc["numa"]["numa_node"], int)
    assert isinstance(pc["numa"]["staging_node"], int)
    print(json.dumps({"strong_stream": sub["value"], "weak": line["value"], "pcie": pc}))
