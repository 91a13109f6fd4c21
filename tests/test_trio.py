"""The lane-trio point operations (ec26_trio.h) on the CPU: tests/cpp/trio_test.cpp runs one 16-lane DPP
row as 16 lockstep threads (DPP fetches and wave votes are barriers) with FE26_CHECK magnitude
assertions on every lane, and compares every trio's doublings / mixed additions with CurveK1x,
including P = Q, P = -Q and P = infinity."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trio_ops_match_one_lane(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not found")
    exe = str(tmp_path / "trio_test")
    subprocess.run([cxx, "-O1", "-std=c++17", "-pthread", "-Wall", "-Wextra", "-Wno-unknown-pragmas", "-Werror",
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "trio_test.cpp")], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("trio ok"), out.stdout
