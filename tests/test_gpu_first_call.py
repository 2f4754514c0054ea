"""First-call latency.  A JVM pays a context's first call once per context: the runtime loads a
kernel file's code object at the first launch of any kernel in it, and the scan's buffers are allocated at first use.
rsh_ctx_create now does both (capi.cpp ctx_warm), so the first scan on a fresh context costs what the next ones do.

The check runs in a fresh process (java-rsync_amd/tools/first_call.py): in this one, other tests have loaded the code
objects already."""
import json
import os
import statistics
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_first_step_on_a_fresh_context_costs_what_the_next_ones_do():
    """rsh_ctx_create in a new process, then BASELINE config 5 as written (16 GiB, B = 131072, dl = 4, every other
    block of the basis replaced; the device-resident Generator + Sender step) five times: the first step within 10 %
    of the median of the other four (+ 0.2 ms for the host timer and the Python calls around it)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "java-rsync_amd", "tools", "first_call.py"), "--only", "5",
                        "--reps", "5"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    steps = out["config5_half_step_ms"]
    rest = statistics.median(steps[1:])
    assert steps[0] <= 1.10 * rest + 0.2, out
