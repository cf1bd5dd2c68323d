"""The N > 1 bench's stage markers and watchdog (vigor_amd/watchdog.py) on
the CPU: two gloo ranks in separate processes, as bench.py --gpus 2 runs them.
With an injected stall (rank 1 sleeps inside a "segment" while rank 0 waits
in a collective) both watchdogs fire: each rank aborts, rank 0 prints the
partial JSON line naming the stage reached, and both exit with status 3.
Without a stall both ranks finish normally. The GPU rehearsal of the same
(bench.py --gpus 2 with VIGPATH_COMM=host and VIGPATH_STALL) runs on the
box (tools/sessions/gpu_r05*.sh)."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

import vigor_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    import torch.distributed as dist
    from vigor_amd.watchdog import Watchdog
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    stall = float(os.environ.get("STALL_S", "0"))
    aborted = []
    wd = Watchdog(rank, world, float(os.environ["BUDGET_S"]),
                  partial={{"metric": "m", "unit": "Mpps"}},
                  abort=lambda: sys.stderr.write("abort r%d\\n" % rank)).start()
    wd.stage("comm init (gloo)")
    dist.init_process_group("gloo")
    for k in range(3):
        wd.stage("timed: step %d/3" % (k + 1))
        if rank == 1 and k == 1 and stall:
            time.sleep(stall)          # a segment that never ends
        dist.barrier()                 # the batch's collective
    wd.stage("report")
    if rank == 0:
        print('{{"value": 1.0}}', flush=True)
    dist.destroy_process_group()
    wd.stage("done")
    wd.stop()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(text):  # (gloo prints its own lines on stdout)
    return [x for x in text.splitlines() if x.startswith("{")]


def _run_ranks(tmp_path, stall_s, budget_s):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(root=ROOT))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), STALL_S=str(stall_s), BUDGET_S=str(budget_s))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    return [p.returncode for p in procs], outs


def test_watchdog_fires_on_injected_stall(tmp_path):
    rcs, outs = _run_ranks(tmp_path, stall_s=60, budget_s=3)
    assert rcs == [3, 3], (rcs, outs)
    line = json.loads(_json_lines(outs[0][0])[-1])
    assert line["partial"] is True and line["value"] is None
    assert line["stage_reached"] == "timed: step 2/3"
    assert line["stages_done"] == ["comm init (gloo)", "timed: step 1/3"]
    assert line["metric"] == "m" and line["n_gpus"] == 2
    assert "no progress" in line["error"]
    # every rank aborted and said so on stderr; rank 1 prints no JSON line
    for r, (so, se) in enumerate(outs):
        assert "abort r%d" % r in se
        assert "WATCHDOG" in se and "[bench r%d/2" % r in se
    assert _json_lines(outs[1][0]) == []


def test_no_stall_runs_to_the_end(tmp_path):
    rcs, outs = _run_ranks(tmp_path, stall_s=0, budget_s=30)
    assert rcs == [0, 0], (rcs, outs)
    assert [json.loads(x) for x in _json_lines(outs[0][0])] == [{"value": 1.0}]
    for r, (_, se) in enumerate(outs):
        assert "WATCHDOG" not in se
        for st in ("comm init (gloo)", "timed: step 3/3", "report", "done"):
            assert "] %s" % st in se


def test_comm_abort_entry_point():
    L = vigor_amd.lib()
    assert L.vp_comm_abort(None) == -22
    assert "vp_comm_abort" in vigor_amd.EXPORTS
