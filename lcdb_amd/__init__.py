"""lcdb_amd -- MI355X-native (gfx950) Snappy block codec for lcdb.

A drop-in for lcdb's ``src/util/snappy.{c,h}`` (the four ``ldb_snappy_*``
C entry points, exported by ``liblcdb_gpu_snappy.so``) plus a batched,
device-resident API that encodes/decodes tens of thousands of SSTable blocks
per launch.  See DESIGN.md and include/lcdb_gpu_snappy.h.

Submodules:
  snappy  -- the codec (GPU only; raises on import if the library is absent)
  corpus  -- synthetic db_bench-shaped block corpora
  build   -- in-tree build of the native libraries
"""

__version__ = "0.1.0"
