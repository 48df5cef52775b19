"""GPU: the RCCL branch of the multi-process exchange on one MI355X
(VERDICT r4 item 7).  A 1-rank `nccl` process group (RCCL) and a
ShardedMapper with force_exchange=True, so the device exchange runs as on N
GPUs with P = 1: the band's export record, the records' all-gather on the
band's exchange stream (_xstream) over the halo's own communicator
(records_comm="shared", the default) and over a second one ("separate",
rec_group), the device merge (dm_merge_bands / _begin / _end), and the host's
event polling — synchronous and pipelined with overlap on.  Every pass must
equal the oracle's clusters after its own batch.

What this does NOT cover: the halo exchange itself.  With P = 1 the band has
no neighbour, so _halo_dev returns before any RCCL call and
exchange_neighbour_rows posts no send / receive.  The batched RCCL neighbour
send / receive has run only with gloo (tests/test_sharded.py's 4-rank test,
the 2-rank GPU tests and the 8-rank one-GPU rehearsal); between devices it is
unverified until a multi-GPU node runs bench.py --gpus N.

The process group runs in a child process (a fresh interpreter started by
subprocess before it touches the GPU), so the pytest process's own GPU
context and the other tests are unaffected."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r'''
import json, os, socket, sys
sys.path[:0] = [{here!r}, {oracle!r}, {pkg!r}]
import numpy as np
import torch
import torch.distributed as dist

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import cases, oracle
from dm.sharded import ShardedMapper
oracle.build()
out = {{}}
p, batches, amin, inc = cases.world_case(61, 2048, 1536, 0.05, 8, 1024, 6, region_frac=0.6)
om = oracle.OracleMap(p)
expect = []
for poses, ranges in batches:
    om.integrate(poses, ranges, amin, inc)
    expect.append(om.frontiers(want_mask=False, want_labels=False)[2])
def run_mode(sm, mode, bad, out):
    # synchronous exchange (dm_merge_bands)
    for k in range(2):
        sm.integrate(*batches[k], amin, inc)
        fr = sm.frontiers()
        if not np.array_equal(fr.clusters, expect[k]):
            bad.append((mode, "sync", k))
    # pipelined, overlap on, depth 2 (dm_merge_bands_begin / _end)
    sm.set_overlap(True)
    got = []
    for k in range(2, 6):
        sm.integrate(*batches[k], amin, inc)
        if k >= 4:
            got.append((k - 2, sm.frontiers_end()))
        sm.frontiers_begin()
    for j in (4, 5):
        got.append((j, sm.frontiers_end()))
    for k, fr in got:
        if fr is None or not np.array_equal(fr.clusters, expect[k]):
            bad.append((mode, "pipelined", k))
    out["passes"] = len(got) + 2
    out["clusters_last"] = int(len(expect[-1]))
    out["fallbacks"] = out.get("fallbacks", 0) + int(sm.fallbacks)

bad = []
for mode in ("shared", "separate"):
  sm = ShardedMapper(p, rank=0, world_size=1, device=0, group=dist.group.WORLD, timeout=60.0,
                     force_exchange=True, records_comm=mode)
  out["nccl"] = bool(sm._nccl)
  out["dev_path"] = bool(sm._dev_path)
  out["rec_group_backend_" + mode] = dist.get_backend(sm.rec_group)
  out["rec_group_is_group_" + mode] = sm.rec_group is dist.group.WORLD
  run_mode(sm, mode, bad, out)
  sm.close()
out["bad"] = bad
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
'''


def test_rccl_exchange_one_rank():
    code = CHILD.format(here=HERE, oracle=os.path.join(REPO, "oracle"),
                        pkg=os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd"))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(lines[-1][7:])
    assert res["nccl"] and res["dev_path"], res
    assert res["rec_group_backend_shared"] == "nccl" and res["rec_group_is_group_shared"], res
    assert res["rec_group_backend_separate"] == "nccl" and not res["rec_group_is_group_separate"], res
    assert res["passes"] == 6 and res["clusters_last"] > 0, res
    assert res["bad"] == [] and res["fallbacks"] == 0, res
