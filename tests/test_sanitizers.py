"""Host-side sanitizers: ASan + UBSan over the CPU codec (oracle)
and the product's host-only wire-format code (fec_frame.cpp), driven by
tests/native/san_driver.c.  GPU sanitizers are not available on this pool; the
device path is covered by bounds-checked parity tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_asan_ubsan_codec_and_frames(tmp_path):
    exe = tmp_path / "san_driver"
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all"]
    objs = []
    for src, lang in (("oracle/fec_oracle.c", "c"), ("tests/native/san_driver.c", "c"),
                      ("quic-fec-eps_amd/csrc/fec_frame.cpp", "c++")):
        o = tmp_path / (os.path.basename(src) + ".o")
        cc = "gcc" if lang == "c" else "g++"
        std = ["-std=c11"] if lang == "c" else ["-std=c++17"]
        subprocess.run([cc, *flags, *std, "-c", os.path.join(ROOT, src), "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["g++", *flags, *objs, "-o", str(exe), "-pthread"], check=True)
    # verify_asan_link_order=0: the environment may preload its own library
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitizers ok" in r.stdout


def _build(tmp_path, name, srcs, flags):
    objs = []
    for src in srcs:
        o = tmp_path / (name + "_" + os.path.basename(src) + ".o")
        subprocess.run(["gcc", *flags, "-std=c11", "-c", os.path.join(ROOT, src), "-o", str(o)], check=True)
        objs.append(str(o))
    exe = tmp_path / name
    subprocess.run(["gcc", *flags, *objs, "-o", str(exe), "-pthread"], check=True)
    return exe


SW_SRCS = ("oracle/fec_oracle.c", "oracle/fec_sw_banded.c", "oracle/fec_cpu_simd.c", "tests/native/san_sw_driver.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_asan_ubsan_sliding_window_and_simd(tmp_path):
    """the banded sliding-window decoder (long systems, more than 256
    repairs alive at one column) and the threaded AVX2 / GFNI codec under ASan +
    UBSan, each against the scalar oracle (tests/native/san_sw_driver.c)."""
    exe = _build(tmp_path, "san_sw", SW_SRCS, ["-O1", "-g", "-fno-omit-frame-pointer",
                                                "-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sw sanitizers ok" in r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_tsan_simd_codec_threads(tmp_path):
    """The SIMD codec's worker threads (encode over repairs / windows, decode over
    runs of whole linked systems) under ThreadSanitizer: no data race."""
    exe = _build(tmp_path, "san_sw_tsan", SW_SRCS, ["-O1", "-g", "-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=900)
    if r.returncode != 0 and "FATAL: ThreadSanitizer" in r.stderr and "memory layout" in r.stderr:
        pytest.skip("ThreadSanitizer cannot map its shadow memory on this kernel")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sw sanitizers ok" in r.stdout
