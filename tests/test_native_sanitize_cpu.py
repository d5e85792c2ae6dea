"""ASan + UBSan self-test of the host C++ cores (text, tokenizers, Markov, HTML, JSON), built
without Python so no sanitizer runtime has to be preloaded into the interpreter."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "csrc", "native")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_native_cores_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           os.path.join(NATIVE, "tests", "selftest.cpp"), os.path.join(NATIVE, "html.cpp"),
           os.path.join(NATIVE, "json.cpp"), "-DSYMB_NO_PYTHON", "-I", NATIVE, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    # verify_asan_link_order=0: tolerate libraries an environment preloads ahead of the runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "selftest ok" in p.stdout, p.stderr[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
@pytest.mark.parametrize("prog", ["natsd_selftest", "gateway_selftest"])
def test_native_servers_under_sanitizers(tmp_path, prog, san):
    """The epoll NATS server and the multi-threaded HTTP gateway, driven over real sockets, under
    ASan+UBSan and under ThreadSanitizer (worker threads, stats, start/stop)."""
    exe = str(tmp_path / prog)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", os.path.join(NATIVE, "tests", prog + ".cpp"),
           os.path.join(NATIVE, "json.cpp"), "-DSYMB_NO_PYTHON", "-I", NATIVE, "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "selftest ok" in p.stdout, p.stderr[-3000:]
