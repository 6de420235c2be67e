"""storm_amd — MI355X-native block-checksum engine behind storm's ``blocks`` API.

Scope (BASELINE.json north_star): XXH64 block checksums of
/root/reference/blocks/checksum.go on gfx950, the Merkle pointer-tree levels built
from them, and per-shard roots gathered over RCCL. Submodules:

* ``blocks``   — Go ``blocks`` API mirror (Checksum, BlockChecksum, VerifyChecksum, batches)
* ``layouts``  — storm block structs (pointer, blob, objectlist, spacelist, singularity)
* ``engine``   — device-resident entry points (raw pointers / torch tensors)
* ``commit``   — f1: level-synchronous Cache.Commit of a dirty forest (stormck_commit_device)
* ``dist``     — shard planning and the root all-gather
* ``build``    — in-tree hipcc build of libstormck.so
"""

ABI_VERSION = 7

__all__ = ["ABI_VERSION"]
