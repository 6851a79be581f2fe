"""Wheel packaging (the reference publishes maturin wheels: .github/workflows/publish-pypi.yml:1-49).

Builds a wheel offline, installs it into a scratch prefix, and imports it from outside
the repo. This checks that the compiled host runtime and the ``relayrl_framework`` shim
ship inside the wheel.
"""
import glob
import os
import subprocess
import sys
import zipfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_wheel_builds_installs_and_imports(tmp_path):
    env = dict(os.environ, RRL_BUILD_TARGETS="native")
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", REPO, "--no-deps", "--no-build-isolation",
                        "-w", str(tmp_path / "dist")], env=env, capture_output=True, text=True, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (whl,) = glob.glob(str(tmp_path / "dist" / "relayrl_prototype_amd-*.whl"))
    assert "linux_x86_64" in whl  # platform wheel: it carries .so files
    names = zipfile.ZipFile(whl).namelist()
    assert any(n.endswith("relayrl_prototype_amd/__init__.py") for n in names)
    assert any("relayrl_prototype_amd/_native" in n and n.endswith(".so") for n in names)
    assert any(n.endswith("relayrl_framework/__init__.py") for n in names)
    assert any(n.endswith("entry_points.txt") for n in names)
    assert not any("/csrc/" in n or n.startswith("tests/") for n in names)

    target = tmp_path / "site"
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--target", str(target), whl],
                       capture_output=True, text=True, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    code = ("import relayrl_prototype_amd as r, relayrl_framework as f, relayrl_prototype_amd._native as n;"
            "assert r.__file__.startswith(%r), r.__file__;"
            "assert f.RelayRLAgent is r.RelayRLAgent and f.TrainingServer is r.TrainingServer;"
            "print(n.env_names())" % str(target))
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["PYTHONPATH"] = str(target)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
