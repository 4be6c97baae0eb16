"""Builds librs_simplify.so (HIP, gfx950) and the circom-simplify CLI in-tree."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "librs_simplify.so")
CLI = os.path.join(PKG, "circom-simplify")
SOURCES = ["engine.hip", "r1cs_io.cpp", "synth.cpp", "host_common.cpp"]
HEADERS = ["field.hpp", "kernels.hpp", "frames_wave.hpp", "spec_loop.hpp", "giant_loop.hpp", "output.hpp", "flatten.hpp", "cluster.hpp", "writer.hpp", "comm.hpp", "host_common.hpp", os.path.join("..", "..", "include", "rs_simplify.h")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    if force or _stale(LIB, deps):
        # every kernel without its own __launch_bounds__ is launched with 256 threads: saying so keeps
        # the backend from sizing promoted private arrays in LDS for 1024-thread workgroups (which
        # capped k_nl_fill / k_round_fill at 2 workgroups per CU)
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "--gpu-max-threads-per-block=256",
               "-o", LIB] + [os.path.join(CSRC, s) for s in SOURCES] + [
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    cli_src = os.path.join(CSRC, "cli.cpp")
    if force or _stale(CLI, [cli_src, LIB]):
        cmd = ["g++", "-O2", "-std=c++17", "-o", CLI, cli_src, "-L" + PKG, "-lrs_simplify",
               "-Wl,-rpath,$ORIGIN"]
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
