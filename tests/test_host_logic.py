"""Host-side logic without a GPU: the orphan query of the identifier job's
file_path stand-in (file_identifier_job.rs:245-309 / shallow.rs:121-139),
walked from the cursor with the query's LIMIT."""
import numpy as np


def _naive(t, loc, cursor=None, children_of=None, under=None):
    out = []
    for fid in range(max(1, cursor or 1), len(t) + 1):
        i = fid - 1
        if t.object_id[i] is not None or t.is_dir[i] or t.location_id[i] != loc:
            continue
        mp = t.materialized_path[i]
        if children_of is not None and mp != children_of:
            continue
        if under is not None and not mp.startswith(under):
            continue
        out.append(fid)
    return out


def test_orphan_query_matches_full_scan():
    from spacedrive_amd.file_identifier import FilePaths
    rng = np.random.default_rng(3)
    t = FilePaths()
    dirs = ["/", "/a/", "/a/b/", "/c/"]
    for i in range(3000):
        t.add(int(rng.integers(1, 3)), dirs[int(rng.integers(0, 4))], f"f{i}",
              is_dir=bool(rng.random() < 0.05))
    for fid in rng.choice(np.arange(1, 3001), 900, replace=False):
        t.object_id[int(fid) - 1] = 7          # linked rows (written directly, as a host would)
    for loc in (1, 2):
        for cursor in (None, 1, 17, 1500, 2999, 5000):
            for kw in ({}, {"children_of": "/a/"}, {"under": "/a/"}):
                ref = _naive(t, loc, cursor, **kw)
                assert t.orphans(loc, cursor, **kw) == ref
                for limit in (1, 100, 101):
                    assert t.orphans(loc, cursor, limit=limit, **kw) == ref[:limit]
