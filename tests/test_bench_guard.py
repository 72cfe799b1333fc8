"""bench.py's one JSON line survives a failing or hanging auxiliary leg
(VERDICT r2 item 1): main() runs with a mocked runner (no GPU) in a child
process, and the line still carries the headline, `roofline` and
`cpu_baseline`."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_FAKE = r'''
import sys, time
sys.path.insert(0, sys.argv[1])
import bench

MODE = sys.argv[2]


class Ctx:
    def valu_peak(self, kind=0):
        return 38.7e12


class FakeRunner:
    def __init__(self, args):
        self.args, self.rank, self.world, self.ctx = args, 0, 1, Ctx()
        self.comm, self._cpu_dedup = None, None

    def world_info(self):
        return {"dist_world_size": 1, "devices_visible": 0, "backend": None,
                "exchange": "none (one GPU: local grouping)"}

    def free(self):
        pass

    def drop_samples(self):
        pass

    def shutdown(self):
        pass

    def run_cas(self, steps, warmup):
        if MODE == "cas_raises":
            raise RuntimeError("injected K1 failure")
        job = ({"error": "SdgpuError(-110, 'sdgpu_group_sharded_device: timed out')"}
               if MODE == "job_fails" else {"value": 7.4e7, "ms_per_step": 13.5})
        return {"cas": {"value": 7.5e7, "unit": "files/s", "ms_per_step": 13.3},
                "job": job,
                "kernels": {"cas_leaves": {"avg_ms": 13.0, "launches": 20}},
                "roofline_inputs": {"chunk_blocks": 1, "parents": 0,
                                    "leaf_compressions": 685_757_283, "fold_compressions": 0,
                                    "avg_leaves_s": 0.013, "bytes": 41_884_044_005}}

    def run_single(self):
        return {"generate_cas_id_4KiB_us": 50.0}

    def run_dir(self, steps):
        raise OSError(28, "No space left on device")

    def cpu_baseline(self):
        return {"value": 1.0e6, "unit": "files/s", "cores": 16, "kind": "port"}

    def run_dedup(self, steps, warmup):
        return {"value": 4.7e10, "unit": "rows/s"}

    def run_consumers(self, steps, warmup):
        return {"orphan_remover": {"value": 1.0}}

    def run_staged(self):
        if MODE == "staged_hangs":
            time.sleep(600)
        raise MemoryError("injected: pin_memory of the config-5 pool failed")

    def run_checksum(self, steps, warmup):
        return {"value": 3100.0, "unit": "GB/s"}


bench.main(["--steps", "20", "--warmup", "5", "--deadline", sys.argv[3]], runner_cls=FakeRunner,
           out=sys.stdout)
'''


def _run(mode, deadline="60"):
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", _FAKE, ROOT, mode, deadline], capture_output=True,
                       text=True, timeout=120)
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    return p, lines, time.monotonic() - t0


def test_raising_legs_keep_the_headline():
    p, lines, _ = _run("staged_raises")
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 7.4e7 and d["ms_per_step"] == 13.5
    assert d["roofline"]["bound"] == "valu" and 0 < d["roofline"]["frac"] < 1
    assert d["cpu_baseline"]["kind"] == "port"
    assert "MemoryError" in d["components"]["staged"]["error"]
    assert "No space left" in d["components"]["dir"]["error"]
    assert d["components"]["checksum"]["value"] == 3100.0   # legs after the failure still ran
    assert d["components"]["dedup"]["value"] == 4.7e10
    assert set(d["leg_wall_s"]) >= {"cas", "staged", "checksum", "total"}


def test_hanging_leg_hits_the_deadline():
    p, lines, dt = _run("staged_hangs", deadline="3")
    assert p.returncode == 4, p.stderr[-3000:]  # the line is printed, the exit is not green
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 7.4e7
    assert d["roofline"]["bound"] == "valu" and d["cpu_baseline"]["cores"] == 16
    assert d["incomplete"]["leg"] == "staged"
    assert "deadline" in d["components"]["staged"]["error"]
    assert dt < 60


def test_failed_headline_still_prints_a_line():
    p, lines, _ = _run("cas_raises")
    assert len(lines) == 1, p.stdout
    assert p.returncode == 3
    d = json.loads(lines[0])
    assert d["value"] is None and "injected K1" in d["components"]["cas"]["error"]
    assert d["components"]["checksum"]["value"] == 3100.0


def test_failed_exchange_has_no_headline():
    """The identifier step's exchange fails (e.g. -ETIMEDOUT from a dead peer):
    the line carries NO headline value (K1 alone is a faster subset of the
    step), keeps K1's rate under components.cas and the roofline,
    and the process exits non-zero."""
    p, lines, _ = _run("job_fails")
    assert p.returncode == 3, p.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["value"] is None and "job step failed" in d["headline_note"]
    assert d["components"]["cas"]["value"] == 7.5e7
    assert "timed out" in d["components"]["identifier_job"]["error"]
    assert d["roofline"]["bound"] == "valu" and d["cpu_baseline"]["kind"] == "port"
