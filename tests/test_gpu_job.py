"""GPU: the identifier as the reference runs it -- the resumable job over a
file_path table (file_identifier_job.rs), the shallow light scan (shallow.rs),
BASELINE config 1 on real files, and files that grow between stat and read.
Expected Objects come from the oracle over the whole run (cas ids from the
oracle's path-based generate_cas_id, grouping from its canonical rule with the
library's pre-existing Objects)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 63, 1000, 4096, 20_000, 102_400, 102_401, 150_000, 1 << 20]


def _make_library(root, n=2500, seed=3):
    """Location 1 (files on disk under root/loc1, dirs /, /a/, /a/b/, /c/,
    ~20 % duplicated content, one row whose file is missing, directory rows) and
    location 2 (rows already linked to Objects, some sharing location 1's
    content: the library-wide existing Objects)."""
    from spacedrive_amd.file_identifier import FilePaths
    rng = np.random.default_rng(seed)
    t = FilePaths()
    loc = os.path.join(root, "loc1")
    dirs = ["/", "/a/", "/a/b/", "/c/"]
    for d in dirs[1:]:
        os.makedirs(os.path.join(loc, d.strip("/")), exist_ok=True)
        parent = "/" + "/".join(d.strip("/").split("/")[:-1])
        t.add(1, parent if parent.endswith("/") else parent + "/", d.strip("/").split("/")[-1],
              is_dir=True)
    contents = []
    for i in range(n):
        if contents and rng.random() < 0.2:
            data = contents[rng.integers(0, len(contents))]
        else:
            size = int(SIZES[rng.integers(0, len(SIZES))]) if rng.random() < 0.3 else \
                int(rng.integers(1, 60_000))
            data = O.synth_file_bytes(10_000 + i, 0, size)
            contents.append(data)
        d = dirs[rng.integers(0, len(dirs))]
        name = f"f{i:05d}.bin"
        if i != 2:  # row 2's file is missing: ENOENT, the row stays an orphan
            with open(os.path.join(loc, d.lstrip("/"), name), "wb") as f:
                f.write(data)
        t.add(1, d, name)
    # location 2: 300 rows already identified and linked (other location)
    for j in range(300):
        data = contents[j % len(contents)] if j % 3 == 0 else O.synth_file_bytes(77_000 + j, 0, 5000)
        fid = t.add(2, "/", f"g{j}.bin")
        if len(data):
            p = os.path.join(root, "tmp_g")
            with open(p, "wb") as f:
                f.write(data)
            t.cas_id[fid - 1] = O.cas_id_path(p, len(data))
        t.object_id[fid - 1] = t.next_object_id
        t.next_object_id += 1
    return t, loc


def _expected(t, loc, fids, rank_of):
    """Oracle Objects for the rows `fids` (ranks rank_of[f]); returns
    {fid: ("existing", object id) | ("rank", creator rank)} and the valid set."""
    n = max(rank_of.values()) + 1
    key = np.zeros(n, np.uint64)
    has = np.zeros(n, np.uint8)
    valid = {}
    for f in fids:
        p = os.path.join(loc, t.rel_path(f))
        r = rank_of[f]
        if not os.path.exists(p):
            valid[f] = False
            continue
        valid[f] = True
        size = os.path.getsize(p)
        if size:
            key[r] = np.frombuffer(bytes.fromhex(O.cas_id_path(p, size)), np.uint64)[0]
            has[r] = 1
    ek, eh = [], []
    for c, o in zip(t.cas_id, t.object_id):
        if c is not None and o is not None:
            ek.append(np.frombuffer(bytes.fromhex(c), np.uint64)[0])
            eh.append(o)
    rep = O.group_reps_existing(key, has, 100, np.array(ek, np.uint64), np.array(eh, np.uint32))
    out = {}
    for f in fids:
        if valid[f]:
            v = int(rep[rank_of[f]])
            out[f] = ("existing", v & 0x7FFFFFFF) if v & 0x80000000 else ("rank", v)
    return out, valid


def _check_against_oracle(t_before, t, loc, fids):
    rank_of = {f: i for i, f in enumerate(fids)}
    exp, valid = _expected(t_before, loc, fids, rank_of)
    creator_obj = {}
    for f in fids:
        if valid[f] and exp[f] == ("rank", rank_of[f]):
            creator_obj[rank_of[f]] = t.object_id[f - 1]
    assert len(set(creator_obj.values())) == len(creator_obj)  # one new Object per creator
    for f in fids:
        if not valid[f]:
            assert t.object_id[f - 1] is None and t.cas_id[f - 1] is None
            continue
        kind, v = exp[f]
        want = v if kind == "existing" else creator_obj[v]
        assert t.object_id[f - 1] == want, (f, exp[f])


def _clone(t):
    import copy
    return copy.deepcopy(t)


def test_job_uninterrupted_vs_resumed_vs_oracle(ctx, tmp_path):
    from spacedrive_amd.file_identifier import FileIdentifierJob
    t0, loc = _make_library(str(tmp_path))
    fids = t0.orphans(1)
    # A: uninterrupted, 3 reference chunks per GPU step
    ta = _clone(t0)
    ja = FileIdentifierJob(ta, 1, loc, chunks_per_step=3, ctx=ctx).init()
    meta = ja.run()
    ja.close()
    assert ja.step_number == ja.task_count == -(-len(fids) // 100)
    # B: 2 GPU steps, state through JSON, a new job (new index) resumes
    tb = _clone(t0)
    jb = FileIdentifierJob(tb, 1, loc, chunks_per_step=3, ctx=ctx).init()
    jb.run(max_steps=2)
    state = json.loads(json.dumps(jb.state()))
    jb.close()
    del jb
    jr = FileIdentifierJob.resume(tb, state, ctx=ctx)
    jr.run()
    jr.close()
    assert ta.object_id == tb.object_id and ta.cas_id == tb.cas_id
    # C: one chunk per step, as the reference runs it
    tc = _clone(t0)
    jc = FileIdentifierJob(tc, 1, loc, chunks_per_step=1, ctx=ctx).init()
    jc.run()
    jc.close()
    assert tc.object_id == ta.object_id
    _check_against_oracle(t0, ta, loc, fids)
    assert meta.total_objects_linked > 300 and meta.total_objects_created > 1000
    assert ta.object_id[fids[2] - 1] is None  # the missing file stays an orphan


@pytest.mark.parametrize("seed", range(3))
def test_job_resumed_at_random_points(ctx, tmp_path, seed):
    """The job paused and resumed from its JSON state several times at random
    step counts, with a random number of reference chunks per GPU step, in a
    fresh job (and a fresh Object index) each time: the table ends equal to
    the uninterrupted run's and to the oracle's Objects
    (file_identifier_job.rs:32-309: the cursor and the counts carry over)."""
    from spacedrive_amd.file_identifier import FileIdentifierJob
    rng = np.random.default_rng(500 + seed)
    t0, loc = _make_library(str(tmp_path), n=1800, seed=40 + seed)
    fids = t0.orphans(1)
    per = int(rng.choice([1, 2, 5]))  # >= 4 GPU steps over ~19 chunks
    ta = _clone(t0)
    ja = FileIdentifierJob(ta, 1, loc, chunks_per_step=per, ctx=ctx).init()
    ja.run()
    ja.close()
    tb = _clone(t0)
    job = FileIdentifierJob(tb, 1, loc, chunks_per_step=per, ctx=ctx).init()
    legs = 0
    while True:
        job.run(max_steps=int(rng.integers(1, 3)))
        state = json.loads(json.dumps(job.state()))
        done = job.step_number >= job.task_count
        job.close()
        legs += 1
        if done:
            break
        job = FileIdentifierJob.resume(tb, state, ctx=ctx)
    assert legs >= 2
    assert tb.object_id == ta.object_id and tb.cas_id == ta.cas_id
    _check_against_oracle(t0, tb, loc, fids)


def test_job_sub_path_and_early_finish(ctx, tmp_path):
    from spacedrive_amd.file_identifier import EarlyFinish, FileIdentifierJob
    t0, loc = _make_library(str(tmp_path), n=800)
    t = _clone(t0)
    job = FileIdentifierJob(t, 1, loc, sub_path="a", chunks_per_step=2, ctx=ctx).init()
    job.run()
    job.close()
    fids = t0.orphans(1, under="/a/")
    _check_against_oracle(t0, t, loc, fids)
    assert all(t.object_id[f - 1] is None for f in t0.orphans(1) if f not in set(fids))
    with pytest.raises(EarlyFinish):  # a location without orphans
        FileIdentifierJob(t, 3, loc, ctx=ctx).init()


def test_shallow_identifier_one_directory(ctx, tmp_path):
    from spacedrive_amd.file_identifier import shallow
    t0, loc = _make_library(str(tmp_path), n=900)
    t = _clone(t0)
    shallow(t, 1, loc, "a", chunks_per_step=4, ctx=ctx)
    fids = t0.orphans(1, children_of="/a/")
    _check_against_oracle(t0, t, loc, fids)
    others = [f for f in t0.orphans(1) if f not in set(fids)]
    assert others and all(t.object_id[f - 1] is None for f in others)  # /a/b/ untouched
    assert shallow(t, 1, loc, "a", ctx=ctx).total_objects_created == 0  # nothing left


def test_config1_directory_bit_exact(ctx, tmp_path):
    """BASELINE config 1: the 10 k-file directory (1 KiB-10 MiB, sparse) through
    sdgpu_identify_files, every cas_id vs the oracle's path-based
    generate_cas_id, plus the grouping with 200 duplicated files."""
    import shutil
    from spacedrive_amd import corpus, dedup
    from spacedrive_amd import file_identifier as fi
    paths, sizes = corpus.write_config1_dir(str(tmp_path / "cfg1"), 10_000, seed=1)
    for i in range(200):  # duplicates: same content, later ids
        d = str(tmp_path / "cfg1" / f"dup{i:03d}.bin")
        shutil.copyfile(paths[i * 37], d)
        paths.append(d)
    sizes = np.array([os.path.getsize(p) for p in paths], np.uint64)
    res = fi.identify(paths, sizes=sizes, ctx=ctx)
    assert np.all(res.status == 0) and np.all(res.has_key == 1)
    got = res.cas_ids()
    for p, s, g in zip(paths, sizes.tolist(), got):
        assert g == O.cas_id_path(p, s), p
    from spacedrive_amd.cas import keys_of
    key = keys_of(res.cas8)
    rep = dedup.group_reps(key, res.has_key, 100, ctx)
    np.testing.assert_array_equal(rep, O.group_reps(key, res.has_key, 100))
    assert np.count_nonzero(rep != np.arange(rep.size)) == 200


def test_file_grown_between_stat_and_read(ctx, tmp_path):
    """A file of at most 100 KiB at stat time that is longer at read time:
    fs::read hashes the whole current content (cas.rs:27-29) -- no -EFBIG,
    including a message longer than any cas message (> 102 408 B)."""
    from spacedrive_amd import cas
    from spacedrive_amd import file_identifier as fi
    cases = [(5000, 20_000), (50_000, 300_000), (102_400, 102_400 + 4096 + 1), (10, 10)]
    paths = []
    for i, (stat_size, real) in enumerate(cases):
        p = tmp_path / f"g{i}"
        p.write_bytes(O.synth_file_bytes(500 + i, 0, real))
        paths.append(str(p))
    res = fi.identify(paths, sizes=np.array([c[0] for c in cases], np.uint64), ctx=ctx)
    assert np.all(res.status == 0)
    for p, (stat_size, _), g in zip(paths, cases, res.cas_ids()):
        assert g == O.cas_id_path(p, stat_size)
        assert cas.generate_cas_id(p, stat_size, ctx) == g


def test_job_sizes_are_fresh_at_identification(ctx, tmp_path):
    """the job passes no stored size; the library stats
    every path when it identifies it (the reference's fresh fs::metadata,
    file_identifier/mod.rs:65,80-81).  Files changed between the job's orphan
    query and the step -- emptied (cas_id None), grown past the 100 KiB
    sampling threshold, shrunk below it, deleted (ENOENT: the row stays an
    orphan) -- get the oracle's Objects for their content at that moment."""
    from spacedrive_amd.file_identifier import FileIdentifierJob
    t0, loc = _make_library(str(tmp_path), n=400, seed=11)
    fids = t0.orphans(1)
    ta = _clone(t0)
    job = FileIdentifierJob(ta, 1, loc, chunks_per_step=2, ctx=ctx).init()
    changed = {}
    for k, f in enumerate(fids[5:45]):
        p = os.path.join(loc, t0.rel_path(f))
        if not os.path.exists(p):
            continue
        mode = k % 4
        if mode == 0:
            open(p, "wb").close()
        elif mode == 1:
            with open(p, "wb") as fh:
                fh.write(O.synth_file_bytes(900 + k, 0, 150_000 + k))
        elif mode == 2:
            with open(p, "wb") as fh:
                fh.write(O.synth_file_bytes(950 + k, 0, 777 + k))
        else:
            os.remove(p)
        changed[f] = mode
    assert len(set(changed.values())) == 4
    job.run()
    job.close()
    _check_against_oracle(t0, ta, loc, fids)
    for f, mode in changed.items():
        if mode == 0:
            assert ta.cas_id[f - 1] is None and ta.object_id[f - 1] is not None
        elif mode == 3:
            assert ta.object_id[f - 1] is None


def test_identify_stats_paths_itself(ctx, tmp_path):
    """identify(paths) with no sizes: sdgpu_identify_files(size = NULL) stats
    in its read pool -- cas ids equal the oracle's at the current sizes, a
    missing path is -ENOENT and an empty file has no cas_id."""
    import errno
    from spacedrive_amd import file_identifier as fi
    sizes = [0, 1, 4096, 102_400, 102_401, 250_000]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"s{i}"
        p.write_bytes(O.synth_file_bytes(1200 + i, 0, s))
        paths.append(str(p))
    paths.append(str(tmp_path / "missing"))
    res = fi.identify(paths, ctx=ctx)
    assert res.sizes is None
    assert res.status[-1] == -errno.ENOENT and res.has_key[-1] == 0
    ids = res.cas_ids()
    for p, s, g in zip(paths, sizes, ids):
        assert g == (O.cas_id_path(p, s) if s else None)
