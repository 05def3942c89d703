"""Guard: nothing that travels to the GPU box may carry a GPU-sanitizer or XNACK build flag.

Round 3's driver GPU test run was refused because `tools/asan/build.sh` linked with a bare
sanitizer flag (no `-Xarch_host`, no `-fno-gpu-sanitize`) and the script was pushed to the
box. This test walks every file the snapshot would carry (repo minus `.gpurunignore`) and
fails on any such flag in sources, scripts and build files; in files that stay behind it
still requires every sanitizer flag to be host-only. The flag strings are assembled at run
time so this file names none of them literally (it is gpurun-ignored as well).
"""
import fnmatch
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = "-f" + "sanitize="
XN = ["xnack" + "+", "HSA_" + "XNACK"]
SCALAR = ["s_" + "store_", "s_" + "buffer_store", "s_" + "atomic_", "s_" + "dcache_wb",
          "s_" + "dcache_discard"]
TEXT_EXT = {".py", ".sh", ".cpp", ".hip", ".h", ".c", ".cc", ".hpp", ".s", ".S", ".ll",
            ".mk", ".cfg", ".toml", ".ini", ".txt", ".json", ".yaml", ".yml"}
ALWAYS_SKIP = {".git", "gpurun_out", "__pycache__", ".pytest_cache"}


def _ignore_patterns():
    pats = []
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                pats.append(line)
    return pats


def _ignored(rel, pats):
    """tar --exclude semantics, as gpurun documents them: './x' anchors at the top,
    a bare name matches at any depth (any path component or trailing sub-path)."""
    parts = rel.split("/")
    for p in pats:
        if p.endswith("/"):
            continue
        if p.startswith("./"):
            q = p[2:]
            for i in range(1, len(parts) + 1):
                if fnmatch.fnmatchcase("/".join(parts[:i]), q):
                    return True
        else:
            for i in range(len(parts)):
                for j in range(i + 1, len(parts) + 1):
                    if fnmatch.fnmatchcase("/".join(parts[i:j]), p):
                        return True
    return False


def _walk():
    pats = _ignore_patterns()
    for d, dirs, files in os.walk(ROOT):
        reld = os.path.relpath(d, ROOT)
        reld = "" if reld == "." else reld
        dirs[:] = [x for x in dirs if x not in ALWAYS_SKIP]
        for fn in files:
            rel = os.path.join(reld, fn) if reld else fn
            ext = os.path.splitext(fn)[1]
            if ext not in TEXT_EXT and fn not in ("Makefile", "makefile"):
                continue
            yield rel, _ignored(rel, pats)


def _host_only(line):
    toks = line.split()
    for i, t in enumerate(toks):
        if t.startswith(SAN):
            host = i > 0 and toks[i - 1] == "-Xarch_host"
            nogpu = "-fno-gpu-sanitize" in toks and not any(x.startswith("-Xarch_") for x in toks)
            if not (host or nogpu):
                return False
    return True


def test_ignore_matcher():
    pats = ["./tools/asan", "__pycache__", "*.log", "./profiles/r0*"]
    assert _ignored("tools/asan/build.sh", pats)
    assert _ignored("a/b/__pycache__/x.pyc", pats)
    assert _ignored("gpurun_out/x/y.log", pats)
    assert _ignored("profiles/r03a_ops.txt", pats)
    assert not _ignored("profiles/traffic.json", pats)
    assert not _ignored("tests/tools/asan/x", pats)


def test_no_gpu_sanitizer_or_xnack_in_travelling_files():
    bad = []
    for rel, ign in _walk():
        try:
            text = open(os.path.join(ROOT, rel), errors="replace").read()
        except OSError:
            continue
        if ign:
            for ln in text.splitlines():
                if SAN in ln and not _host_only(ln) and not ln.lstrip().startswith(("#", '"', "'", "//")):
                    bad.append((rel, "non-host sanitizer flag", ln.strip()[:120]))
            continue
        if SAN in text:
            bad.append((rel, "sanitizer flag in a travelling file", ""))
        for x in XN:
            if x in text:
                bad.append((rel, "xnack setting", x))
        if os.path.splitext(rel)[1] in (".hip", ".cpp", ".h", ".s", ".S", ".ll", ".c"):
            for x in SCALAR:
                if re.search(re.escape(x), text):
                    bad.append((rel, "scalar-cache write", x))
    assert not bad, bad
