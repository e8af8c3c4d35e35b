"""CPU tests of bench.py's rank launcher (the driver's
`python bench.py --gpus N` runs): without an outer torch.distributed.run,
--gpus N starts N rank processes itself and rank 0's line reports n_gpus = N;
a WORLD_SIZE that disagrees with --gpus is an error.  --dry-protocol runs the
rank protocol (gloo barrier, MAX over ranks) with no GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--steps", "3", "--warmup", "1", "--dry-protocol"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == n and line["steps"] == 3 and line["warmup"] == 1
    pids = line["rank_pids"]
    assert len(pids) == n and len(set(pids)) == n
    # the launching process is none of the ranks
    assert all(isinstance(p, int) for p in pids)


def test_single_rank_runs_in_process():
    r = _run(["--gpus", "1", "--steps", "2", "--warmup", "0", "--dry-protocol"])
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _lines(r.stdout)
    assert line["n_gpus"] == 1 and len(line["rank_pids"]) == 1


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "4", "--dry-protocol"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
    assert not _lines(r.stdout)



def test_post_merge_open_merge_finished_record():
    """The post-merge open leg's merge-finished record (bench._record_bytes) is
    EncodeLogRecord of {MergeFinishedKey, strconv.Itoa(nonMergeFileId)}
    (merge.go:154-168), byte for byte the golden generator's encoding, and
    the oracle decodes it back."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    import make_golden as mg
    from oracle import cly_oracle as co
    for v in (b"0", b"128", b"4096", b"1000000"):
        rec = bench._record_bytes(mg.MERGE_FIN_KEY, v)
        assert rec == mg.encode_record(mg.MERGE_FIN_KEY, v)
        t, st, end = co.scan_file(np.frombuffer(rec, np.uint8).copy(), 0)
        assert len(t) == 1 and end == len(rec) and int(t["value_size"][0]) == len(v)
