"""CPU tests of host-side native code (no GPU): the pread pool behind
vx_verify_files (vortex_amd/csrc/vx_files.hpp), stressed with back-to-back
generations whose item vector is rebuilt between runs (and the pipelined
start/wait form), plain, under ThreadSanitizer and under ASan+UBSan (host
code only, as the GPU pool allows)."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "native", "readers_stress.cpp")


@pytest.mark.parametrize("sanitize", [None, "thread", "address,undefined"])
def test_reader_pool_generations(tmp_path, sanitize):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path / ("rs_" + (sanitize or "plain").replace(",", "_"))
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "vortex_amd", "csrc"), SRC, "-o", str(exe), "-lpthread"]
    if sanitize:
        cmd.insert(1, "-fsanitize=" + sanitize)
        if "undefined" in sanitize:
            cmd.insert(2, "-fno-sanitize-recover=undefined")
    subprocess.run(cmd, check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    out = subprocess.run([str(exe), str(tmp_path / "scratch.bin"), "1500", "6"], capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["errors"] == 0


def _segments_dump(tmp_path):
    exe = tmp_path / "segments_dump"
    if not exe.exists():
        subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "vortex_amd", "csrc"),
                        os.path.join(ROOT, "tests", "native", "segments_dump.cpp"), "-o", str(exe)], check=True)
    return exe


def _run_dump(exe, lens, pl, check_every=0):
    out = subprocess.run([str(exe), str(pl), str(check_every)], input="\n".join(map(str, lens)) + "\n",
                         capture_output=True, text=True, timeout=300, check=True).stdout
    text, summary = out.rsplit("\n", 2)[0] + "\n", json.loads(out.rstrip("\n").rsplit("\n", 1)[1])
    return text, summary


def test_segment_walk_matches_geometry_on_reference_layouts(tmp_path, golden):
    """The engine's piece -> file-segment map (vx_files.hpp, binary search for
    the first overlapping file) equals the geometric interval intersection on
    all of file_store.rs's layouts and the integration geometries, in both
    file orders, and the reference's own filter-every-file walk on every piece."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import interval_segments, interval_segments_sweep, segments_text

    exe = _segments_dump(tmp_path)
    assert len(golden["file_store_layouts"]) >= 17
    for e in golden["file_store_layouts"]:
        for lens in ([f["len"] for f in e["files"]], [f["len"] for f in e["files"]][::-1]):
            pl = e["piece_length"]
            geo = interval_segments(lens, pl)
            assert interval_segments_sweep(lens, pl) == geo, e["name"]
            text, summary = _run_dump(exe, lens, pl, check_every=1)
            assert text == segments_text(geo), e["name"]
            assert summary["linear_checked"] == summary["pieces"] and summary["linear_mismatches"] == 0


def test_segment_walk_100k_files(tmp_path, golden):
    """10^5 files, 145,358 pieces of 16 KiB (make_golden.many_files_layout):
    the segment table equals the committed geometric one, every 97th piece
    equals the reference's filter-every-file walk (file_store.rs:238-241), and
    mapping all pieces stays far from quadratic (the per-piece walk over every
    file is ~1.5e10 file checks here)."""
    import hashlib
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import many_files_lens

    want = golden["many_files_layout"]
    lens = many_files_lens()
    assert hashlib.sha1(" ".join(map(str, lens)).encode()).hexdigest() == want["files_sha1"]
    text, summary = _run_dump(_segments_dump(tmp_path), lens, want["piece_length"], check_every=97)
    assert summary["pieces"] == want["num_pieces"] and summary["files"] == want["nfiles"]
    assert hashlib.sha1(text.encode()).hexdigest() == want["segments_text_sha1"]
    assert summary["linear_checked"] >= want["num_pieces"] // 97 and summary["linear_mismatches"] == 0
    assert summary["build_ms"] < 2000, summary  # ~40 ms measured here (the filter-every-file walk: seconds)


def _disk_dir(tmp_path):
    """A directory on a filesystem that takes O_DIRECT (not tmpfs), or None."""
    for d in (str(tmp_path), "/var/tmp", os.path.join(ROOT, "build")):
        try:
            os.makedirs(d, exist_ok=True)
            p = os.path.join(d, ".vx_odirect_probe")
            with open(p, "wb") as f:
                f.write(b"\0" * 8192)
            fd = os.open(p, os.O_RDONLY | os.O_DIRECT)
            os.close(fd)
            os.unlink(p)
            return d
        except OSError:
            continue
    return None


def test_direct_reads_of_uncached_ranges(tmp_path):
    """vx_files::DirectIo (the re-verify's O_DIRECT path):
    every read returns the file's bytes whatever the alignment; with it
    enabled (vx_config.direct_io = 1) ranges not in the page cache go O_DIRECT
    (mincore probe) and cached ones do not; a file sampled as (nearly) all
    cached is read buffered with no per-read probe; disabled, nothing goes
    direct.  resident_fraction (sampled once per call; it picks the re-verify's
    cold chunk) is ~0 on the evicted file, ~0.5 half cached, 1 on the cached
    one, and 1 when nothing is mapped.  A file
    renamed over the path after it was opened does not leak into the reads:
    the direct descriptor reopens the open file."""
    d = _disk_dir(tmp_path)
    if d is None:
        pytest.skip("no filesystem here takes O_DIRECT")
    exe = tmp_path / "direct_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "vortex_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "direct_check.cpp"), "-o", str(exe)], check=True)
    path = os.path.join(d, f"vx_direct_{os.getpid()}.bin")
    try:
        with open(path, "wb") as f:
            f.write(os.urandom((8 << 20) + 12345))
            f.flush()
            os.fsync(f.fileno())

        def run(mode, evict, replacement=None):
            fd = os.open(path, os.O_RDONLY)
            if evict:
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            if evict == "half":  # only the first half cached: the file is probed per read
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)  # no readahead past the half
                os.pread(fd, (8 << 20) // 2, 0)
            elif not evict:
                while os.read(fd, 1 << 20):  # fault every page in
                    pass
            os.close(fd)
            extra = [replacement] if replacement else []
            out = subprocess.run([str(exe), path, str(mode)] + extra, capture_output=True, text=True, check=True,
                                 timeout=60)
            res = json.loads(out.stdout)
            assert res["reads"] >= 9 and res["mismatches"] == 0, res
            resident.append(res["resident"])
            return res["direct_bytes"]

        resident = []
        assert run(0, evict=True) == 0 and resident[-1] == 1.0  # nothing mapped: the warm choice stands
        cold = run(1, evict=True)
        assert resident[-1] < 0.5, resident  # the kernel may keep a few pages
        warm = run(1, evict=False)
        assert resident[-1] == 1.0
        assert warm == 0  # cached: buffered
        # evicted pages read direct (the kernel may keep a few pages; most ranges go direct)
        assert cold > 0
        # half cached: below the warm threshold, so each read is probed; the cached half stays buffered
        half = run(1, evict="half")
        assert 0.3 < resident[-1] < 0.9, resident
        assert 0 < half < cold
        # a small file of a large torrent, its first 80 % cached: with 2 residency samples
        # (both in the cached part) it looked all cached and nothing went direct; with the per-file
        # minimum it is probed per read, so the uncached tail's aligned ranges go O_DIRECT
        big = path + ".big"
        with open(big, "wb") as f:
            f.truncate(1 << 30)  # sparse: only its share of the samples matters
        try:
            fd = os.open(path, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)
            os.pread(fd, int((8 << 20) * 0.8) & ~4095, 0)
            os.close(fd)
            out = subprocess.run([str(exe), path, "2", big], capture_output=True, text=True, check=True, timeout=60)
            res = json.loads(out.stdout)
            assert res["reads"] >= 9 and res["mismatches"] == 0, res
            assert res["direct_bytes"] > 0, res
        finally:
            os.unlink(big)
        # another file renamed over the path after the open: reads still match the opened file
        other = path + ".new"
        with open(other, "wb") as f:
            f.write(os.urandom((8 << 20) + 12345))
            f.flush()
            os.fsync(f.fileno())
        assert run(1, evict=True, replacement=other) > 0  # direct reads happened, and none mismatched
    finally:
        for p in (path, path + ".new"):
            if os.path.exists(p):
                os.unlink(p)
