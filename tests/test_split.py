"""CPU: the self-balancing split's claim word (include/vx_hash.h vx_split).

The split replaces the planned head/tail cut of a bulk re-verify
(torrent.rs:724-740's par_iter, now shared with the engine) with one claim
word: the caller's pool takes pieces from the head (vx_split_claim), the
engine takes groups from the top (split_take_tail, exercised here through the
test build's vx_tuning_split_take_tail).  These tests need no GPU: they drive
the word from the oracle's claim pool (oracle/pool_oracle.cpp, the stand-in
for vortex's rayon threads) and a Python thread playing the engine, and check
that every piece is taken exactly once, the engine's pieces are one
contiguous tail, and the pool's verdicts are check_piece_hash_sync's.
"""
import ctypes
import hashlib
import os
import random
import subprocess
import threading

import pytest

import oracle
from conftest import ROOT


def _layout(tmp_path, pl, sizes, seed=7):
    paths = []
    for k, L in enumerate(sizes):
        p = tmp_path / f"f{k}.bin"
        p.write_bytes(oracle.gen_piece(seed, k, L))
        paths.append(str(p))
    data = b"".join(open(p, "rb").read() for p in paths)
    exp = b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))
    return paths, exp


def test_split_struct_matches_header(tmp_path):
    """ctypes' vx_split has the C layout (offsets and size)."""
    from vortex_amd import _lib

    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vx_hash.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(vx_split),'
                   ' offsetof(vx_split, pool_done), offsetof(vx_split, start_ns), offsetof(vx_split, first),'
                   ' offsetof(vx_split, end), offsetof(vx_split, cpu_threads), offsetof(vx_split, cpu_thread_rate),'
                   ' offsetof(vx_split, pool_last_ns));'
                   'return 0;}\n')
    exe = tmp_path / "s"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    S = _lib.vx_split
    assert got == [ctypes.sizeof(S), S.pool_done.offset, S.start_ns.offset, S.first.offset, S.end.offset,
                   S.cpu_threads.offset, S.cpu_thread_rate.offset, S.pool_last_ns.offset]


def test_split_init_validation():
    from vortex_amd import _lib
    from vortex_amd._lib import VX_EINVAL, lib

    s = _lib.vx_split()
    assert lib().vx_split_init(ctypes.byref(s), 5, 4, 1, 0.0) == VX_EINVAL
    assert lib().vx_split_init(ctypes.byref(s), 0, 1 << 32, 1, 0.0) == VX_EINVAL
    assert lib().vx_split_init(ctypes.byref(s), 0, 3, 1, -1.0) == VX_EINVAL
    assert lib().vx_split_init(ctypes.byref(s), 2, 5, 1, 0.0) == 0
    assert [lib().vx_split_claim(ctypes.byref(s)) for _ in range(4)] == [2, 3, 4, -1]
    assert lib().vx_split_boundary(ctypes.byref(s)) == 5  # the engine took nothing
    empty = _lib.vx_split()
    assert lib().vx_split_init(ctypes.byref(empty), 9, 9, 1, 0.0) == 0
    assert lib().vx_split_claim(ctypes.byref(empty)) == -1


def test_pool_alone_takes_every_piece(tmp_path):
    """No engine: the claim pool verifies [first, end) like the plain pool."""
    from vortex_amd.hash_pool import Split

    pl = 4096
    paths, exp = _layout(tmp_path, pl, [3 * pl + 5, 0, 7 * pl, pl // 2 + 1])
    n = len(exp) // 20
    with open(paths[2], "r+b") as f:
        f.seek(pl + 9)
        f.write(b"\xee")
    sp = Split(0, n, cpu_threads=3)
    taken = oracle.pool_verify_files_claim(paths, [os.path.getsize(p) for p in paths], pl, exp, 3, sp.claim_fn,
                                           sp.done_fn, sp.arg, 0, sp.matched)
    assert taken == n and sp.pool_done == n and sp.boundary == n
    assert sp.s.start_ns <= sp.s.pool_last_ns  # the pool's last verdict time (the engine's balance sample)
    assert sp.verdicts() == oracle.pool_verify_files(paths, [os.path.getsize(p) for p in paths], pl, exp)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_claims_from_both_ends_race(tmp_path, seed):
    """The pool's threads claim from the head while an engine thread takes
    random groups from the top, both as fast as they can: every piece goes to
    exactly one side, the engine's groups tile one contiguous tail, the pool's
    pieces are [first, boundary), and the pool's verdicts (one damaged piece
    on its side, a truncated last file) match the plain pool's."""
    from vortex_amd import _lib
    from vortex_amd.hash_pool import Split

    rng = random.Random(seed)
    pl = 1024
    sizes = [rng.randint(1, 40) * pl + rng.randint(0, pl - 1) for _ in range(6)]
    paths, exp = _layout(tmp_path, pl, sizes, seed)
    n = len(exp) // 20
    first = rng.randint(0, 3)
    with open(paths[0], "r+b") as f:  # damage piece first+1 (the head: the pool's side)
        f.seek((first + 1) * pl + 3)
        f.write(b"\x00\x01")
    lens = [os.path.getsize(p) for p in paths]
    os.truncate(paths[-1], max(0, lens[-1] - pl - 7))  # the last file short: its pieces are I/O errors
    sp = Split(first, n, cpu_threads=4)
    tuning = _lib.tuning()
    groups = []

    def engine():
        stop = n
        while True:
            was = ctypes.c_uint64()
            new = tuning.vx_tuning_split_take_tail(ctypes.byref(sp.s), rng.randint(1, 9), ctypes.byref(was))
            assert was.value == stop  # the only engine: the stop is where it left it
            if new == stop:
                break
            groups.append((new, stop))
            stop = new

    th = threading.Thread(target=engine)
    th.start()
    taken = oracle.pool_verify_files_claim(paths, lens, pl, exp, 4, sp.claim_fn, sp.done_fn, sp.arg, first,
                                           sp.matched)
    th.join()
    b = sp.boundary
    assert taken == b - first and sp.pool_done == taken
    tiled = b
    for lo, hi in reversed(groups):  # the engine's groups, from the boundary up, no gap, no overlap
        assert lo == tiled
        tiled = hi
    assert tiled == n
    want = oracle.pool_verify_files(paths, lens, pl, exp)
    assert sp.verdicts()[:b - first] == want[first:b]


_ATTACH_CHILD = r"""
import ctypes, mmap, os, sys
sys.path.insert(0, sys.argv[1])
import oracle
from vortex_amd import _lib
from vortex_amd.hash_pool import Split
role, shm, n, pl = sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
paths, lens = sys.argv[6].split(','), [int(x) for x in sys.argv[7].split(',')]
exp = bytes.fromhex(open(sys.argv[8]).read())
fd = os.open(shm, os.O_RDWR)
mm = mmap.mmap(fd, ctypes.sizeof(_lib.vx_split) + n)
os.close(fd)
sp = Split.attach(mm, 0, n, False)
if role == "pool":
    print(oracle.pool_verify_files_claim(paths, lens, pl, exp, 3, sp.claim_fn, sp.done_fn, sp.arg, 0, sp.matched))
else:  # an engine stand-in: groups from the top, verified with the oracle
    allv = oracle.pool_verify_files(paths, lens, pl, exp, threads=2)
    t = _lib.tuning()
    taken = 0
    while True:
        was = ctypes.c_uint64()
        lo = t.vx_tuning_split_take_tail(ctypes.byref(sp.s), 5, ctypes.byref(was))
        if lo >= was.value:
            break
        for i in range(lo, was.value):
            sp.matched[i] = b"\x01" if allv[i] else b"\x00"
        taken += was.value - lo
    print(taken)
sp = None
mm.close()
"""


def test_split_shared_across_processes(tmp_path):
    """The /dev/shm form of the split (Split.attach; bench.multi_balanced at
    N > 1): a claim pool in one process and two engine stand-ins in two
    others claim from one word and write one verdict array; every piece is
    taken once and every verdict is the plain pool's."""
    import mmap

    from vortex_amd import _lib
    from vortex_amd.hash_pool import Split

    pl = 2048
    paths, exp = _layout(tmp_path, pl, [40 * pl + 3, 7, 55 * pl], seed=21)
    lens = [os.path.getsize(p) for p in paths]
    n = len(exp) // 20
    with open(paths[2], "r+b") as f:
        f.seek(9 * pl)
        f.write(b"\xab")
    want = oracle.pool_verify_files(paths, lens, pl, exp)
    shm = tmp_path / "split.shm"
    size = ctypes.sizeof(_lib.vx_split) + n
    shm.write_bytes(bytes(size))
    fd = os.open(shm, os.O_RDWR)
    mm = mmap.mmap(fd, size)
    os.close(fd)
    Split.attach(mm, 0, n, True, 3, 0.0, engines=2)
    (tmp_path / "exp.hex").write_text(exp.hex())
    args = [ROOT, str(shm), str(n), str(pl), ",".join(paths), ",".join(map(str, lens)), str(tmp_path / "exp.hex")]
    procs = [subprocess.Popen([os.sys.executable, "-c", _ATTACH_CHILD, args[0], role] + args[1:],
                              stdout=subprocess.PIPE, text=True) for role in ("engine", "pool", "engine")]
    taken = [int(p.communicate(timeout=240)[0].split()[-1]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    sp = Split.attach(mm, 0, n, False)
    assert sum(taken) == n and taken[1] == sp.boundary and sp.pool_done == taken[1]
    assert sp.verdicts() == want
    sp = None
    mm.close()
