"""CPU: the host-side C ABI code (zonos_amd/csrc/capi.cpp -- descriptor validation, the DAC
workspace plan, the step / prefill / hybrid / DAC launch sequences and error propagation) built
with AddressSanitizer + UBSan, every device entry point replaced by a recording stub
(tests/asan/capi_asan.cpp). SURVEY.md §5 "Race detection / sanitizers": the GPU pool refuses
GPU ASAN, so the sanitizer runs on the host code only."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/lib/libamdhip64.so"),
                    reason="needs g++ and the ROCm runtime library")
def test_capi_host_code_under_asan(tmp_path):
    exe = str(tmp_path / "capi_asan")
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-Wall", "-Werror", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=all", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(REPO, "zonos_amd", "csrc", "capi.cpp"), os.path.join(REPO, "tests", "asan", "capi_asan.cpp"),
           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:verify_asan_link_order=0",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "all checks passed" in r.stdout, r.stdout + r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
