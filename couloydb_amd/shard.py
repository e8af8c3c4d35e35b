"""Multi-GPU sharding of the scan.

Records never span files (db.go:376-385), so every file decodes independently
from offset 0: the scan shards by contiguous fid ranges, one range per GPU
(one process per GPU), balanced by bytes, with no collective on the data path.
Each rank returns its tuples; the host concatenates them in fid order, which
is the order db.loadIndex consumes them in (db.go:582, fids ascending) — the
tx buffering (db.go:604-627) stays on the host because a commit marker may
live in a later file, possibly on another rank.
"""


def partition_by_bytes(sizes, nranks):
    """Split files (in fid order, sizes in bytes) into nranks contiguous ranges
    with nearly equal byte totals.  Returns [(lo, hi)] index ranges (hi
    exclusive); empty ranges are allowed when there are fewer files than ranks."""
    n = len(sizes)
    total = float(sum(sizes))
    bounds = [0]
    acc = 0.0
    r = 1
    for i, s in enumerate(sizes):
        # close the current range once it reaches its share of the bytes
        while r < nranks and acc + s / 2.0 > total * r / nranks and bounds[-1] < i:
            bounds.append(i)
            r += 1
        acc += s
    while len(bounds) < nranks:
        bounds.append(n)
    bounds.append(n)
    return [(bounds[k], bounds[k + 1]) for k in range(nranks)]


def shard_for_rank(files, rank, world):
    """files: list of (fid, size) sorted by fid -> this rank's sub-list."""
    lo, hi = partition_by_bytes([s for _, s in files], world)[rank]
    return files[lo:hi]
