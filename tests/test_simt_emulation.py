"""CPU check of the product kernel sources through the SIMT emulation build
(tests/simt): lzma-java_amd/csrc compiled with g++ against emulated HIP
headers (wave width 1), AddressSanitizer + UBSan on, run through the C ABI
against the oracle for 7 parameter sets x 54 ragged inputs. Catches
out-of-bounds accesses and logic errors in mf/enc/dec before a GPU run."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMT = os.path.join(REPO, "tests", "simt")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("form", ["default", "bench_form"])
def test_emulated_kernels_bit_exact_under_asan(form):
    """form: the parser as these small batches run it by default (one wave per stream, the
    literal coders in LDS: few streams per CU); as the 4096-stream bench runs it (literal
    coders in HBM, LZG_ENC_LITLDS=0), on the smaller input set ("tiny")."""
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    mode = "quick"
    if form == "bench_form":
        env["LZG_ENC_LITLDS"], mode = "0", "tiny"
    r = subprocess.run([os.path.join(SIMT, "build", "emu_check"), mode], capture_output=True, text=True,
                       env=env, timeout=600)
    tail = "\n".join((r.stdout + r.stderr).splitlines()[-20:])
    assert r.returncode == 0, tail
    assert "0 failures" in r.stdout, tail
    errors = [l for l in r.stderr.splitlines() if "runtime error" in l and "emu_check.cpp" not in l]
    assert not errors, "\n".join(errors[:10])


@pytest.mark.timeout(900)
def test_emulated_range_coder_exact_replay_path_bit_exact():
    """rc.hip's exact-replay path (taken by a block with a pending run of
    0xFF bytes, about once per 2^16 shifts) built to run for EVERY block
    (LZG_RC_FORCE_REPLAY), bit-exact against the oracle on the same inputs."""
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT, "replay"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(SIMT, "build", "replay", "emu_check"), "quick"], capture_output=True, text=True,
                       env=env, timeout=600)
    tail = "\n".join((r.stdout + r.stderr).splitlines()[-20:])
    assert r.returncode == 0, tail
    assert "0 failures" in r.stdout, tail
