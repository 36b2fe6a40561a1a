"""Host parsers under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/native/Makefile builds the scene-ingest sources (glTF / GLB, scene and rt-box JSON, PNG / JPEG
decode, PLY, torus sampling, capture writers) with -fsanitize=address,undefined
-fno-sanitize-recover=all into a standalone driver (no device code, no LD_PRELOAD: the sanitizer
runtimes are linked into the executable). The driver decodes every committed fixture, then
deterministic mutations of each (byte flips, truncation, extreme integers, span duplication /
deletion, number substitution in the text formats). A mutated file may be accepted or rejected; a
sanitizer report, an escaped C++ exception or any other abort fails the test. Bugs this found and
fixed: over-subscribed JPEG Huffman lengths writing past the lookup table, 32-bit IDCT overflow on
corrupt coefficients, strtod past the end of an unterminated JSON buffer, a directory read as a file
throwing out of the C-ABI, "scenes" dereferenced before validation, a PLY header without a final
newline, misaligned accessor loads.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
FIXTURES = os.path.join(HERE, "golden", "ingest")


@pytest.fixture(scope="module")
def fuzz_bin():
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    r = subprocess.run(["make", "-j8"], cwd=NATIVE, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(NATIVE, "_build", "ingest_fuzz")


@pytest.mark.parametrize("seed", [0, 1])
def test_parsers_under_asan_ubsan(fuzz_bin, tmp_path, seed):
    r = subprocess.run([fuzz_bin, FIXTURES, str(tmp_path), "400", str(seed)], capture_output=True, text=True,
                       timeout=600, env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                         "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "no sanitizer report" in r.stdout
    print(r.stdout.strip())
