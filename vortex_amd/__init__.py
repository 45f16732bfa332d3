"""vortex_amd — MI355X-native SHA-1 piece-verification engine.

A drop-in for the "Parallel hash computations" pool of Nehliin/vortex
(README.md:44-45; bittorrent/src/peer_comm/peer_connection.rs:1145-1158,
bittorrent/src/torrent.rs:415-442, 724-740).  The product is the HIP library
``libvortex_amd.so`` with the C ABI in ``include/vx_hash.h``; this package is
the Python mirror used by tests and the benchmark.

Modules
  hash_pool  HashPool / DownloadedPiece / verify_pieces (reference names)
  device     device-resident batches on torch tensors (the hot path)
  _lib       ctypes binding (fails loudly when the library is missing)
"""
from ._lib import LIB_PATH, VxError, lib  # noqa: F401

__all__ = ["LIB_PATH", "VxError", "lib"]
