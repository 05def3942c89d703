"""Host-side AddressSanitizer run of the C-ABI (SURVEY.md §5 "Race detection /
sanitizers": `-fsanitize=address` host builds of the C-ABI). GPU ASan is not available on
this pool, so every libisg source is rebuilt with the host half instrumented
(tools/asan/build.sh, -Xarch_host -fsanitize=address) and linked into
tools/asan/abi_host_check.cpp, which drives the argument validation, error plumbing,
executor record parsing / pointer fix-ups and host item-array chunking with valid and
malformed inputs. Any ASan report fails the test. No GPU is needed (launches fail
cleanly without a device)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_abi_host_paths_under_asan():
    out = os.path.join(ROOT, "tools", "asan", "_build")
    b = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan", "build.sh"), out],
                       capture_output=True, text=True, timeout=1200)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23")
    r = subprocess.run([os.path.join(out, "abi_host_check")], capture_output=True, text=True,
                       timeout=300, env=env)
    print(r.stdout)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "OK: 0 failure(s)" in r.stdout
