"""The endpoint-ceiling tools stay runnable (tools/h2_rate.sh, tools/zmtp_rate.sh): an -O2 build of
each self-test and one short run, every message accounted for (profiles/r6_ingest_ceilings_box.txt
holds the measured numbers)."""
import json
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_zmtp_rate_tool():
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "zmtp_rate.sh"), "0.3", "1024"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    rows = _lines(r.stdout)
    assert len(rows) == 6 and all(x["messages"] > 0 for x in rows)
    assert {x["connection_per_message"] for x in rows} == {True, False}


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/conda/include/nghttp2/nghttp2.h"),
                    reason="no host compiler or nghttp2 headers")
def test_h2grpc_rate_tool():
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "h2_rate.sh"), "0.3", "1024"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    rows = _lines(r.stdout)
    assert [x["clients"] for x in rows] == [1, 4, 16, 64] and all(x["ok"] and x["uploads"] > 0 for x in rows)
