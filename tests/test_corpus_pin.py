"""The synthetic workload generator, pinned to lcdb itself.

lcdb_amd/csrc/corpus.c restates db_bench's fillseq entries
(bench/db_bench.c:206-257, src/util/testutil.c:76-103, src/util/random.c:22-55)
packed by the block builder (src/table/block_builder.c:91-151, flushed by
src/table/table_builder.c:251-254).  Here lcdb's own ``ldb_build_table``
(oracle/harness/build_table.c, linked against lcdb's sources with lcdb's
snappy.c) writes a table of the same entries and lcdb's own ``ldb_read_block``
(oracle/harness/dump_blocks.c) reads its data blocks back: every full data
block must equal the generator's block of the same index, byte for byte.
The table's last data block holds the leftover entries (flushed by
``ldb_tablegen_finish``), so it is compared as a prefix only.
"""
from __future__ import annotations

import pytest

from lcdb_amd import corpus
from table_io import LDB_OK, build_table, dump_blocks


@pytest.mark.parametrize("entries,block_size", [(3000, 4096), (3000, 65536), (600, 16384)])
def test_generator_blocks_equal_lcdb_table_blocks(tmp_path, entries, block_size):
    path = build_table(tmp_path, entries, block_size)
    d = dump_blocks(path, str(tmp_path / "dump.bin"), verify=True)
    assert all(rc == LDB_OK for rc in d.rc)
    data = d.n - 2                    # the dump ends with the metaindex and index blocks
    assert data >= 2
    full = data - 1
    gen = corpus.fillseq(data, block_size=block_size)
    for i in range(full):
        assert gen.block(i) == d.contents[i], f"data block {i} of {data} differs"
    # the generator's next block continues the same entries past the table's end
    last = d.contents[full]
    assert len(last) < len(gen.block(full)) or gen.block(full) == last
