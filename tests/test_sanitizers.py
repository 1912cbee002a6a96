"""Host sanitizers ("Race detection / sanitizers"): the CPU oracle — the checker every
parity test trusts — built with AddressSanitizer + UndefinedBehaviorSanitizer (no recovery) and driven
through every exported entry point, fp64 and fp32, including the edge cases the GPU tests use (a ray
with all-zero weights, masked rays, 512 + 512 samples, the 4x128 config-1 network)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], timeout=600)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_build", "oracle_sanitize")], capture_output=True, text=True,
                         timeout=600, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1", OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    assert "runtime error" not in out.stderr and "ERROR: AddressSanitizer" not in out.stderr
    assert "oracle sanitizer run: ok" in out.stdout
