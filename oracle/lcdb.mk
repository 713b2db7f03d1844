# oracle/lcdb.mk -- lcdb compiled from its own sources, in place, to check
# the drop-in end to end (TEST INFRASTRUCTURE ONLY).
#
# Every lcdb library source of CMakeLists.txt:191-241 EXCEPT src/util/snappy.c
# is compiled from $(REF) (flags of CMakeLists.txt:102-127: C89, _GNU_SOURCE,
# pthreads, fdatasync/pread) into _ref/lcdb/liblcdb_core.a.  Each program is
# then linked twice:
#   <name>.cpu  with lcdb's own src/util/snappy.c     (the reference codec)
#   <name>.gpu  with lcdb_amd/liblcdb_gpu_snappy.so  (the drop-in, unchanged
#               callers: table_builder.c, format.c, t-snappy.c ...)
# Programs: lcdb's unchanged test suites that reach the codec (test/t-*.c)
# and our harnesses: harness/build_table.c (config 5) and harness/
# dump_blocks.c (every block of an .ldb as ldb_read_block returns it, the
# pin of the block-framing rows), and harness/build_table_batched.c (config 5
# through the batched lgs_table_* entry points; linked only as .gpu).
# Outputs only in _ref/.
#   make -C oracle -f lcdb.mk        (needs $(REF); the binaries travel)

REF    ?= /root/reference
CC     ?= gcc
HERE   := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
OUT    := $(HERE)_ref/lcdb
GPULIB := $(abspath $(HERE)../lcdb_amd)
CFLAGS := -std=c89 -O2 -D_GNU_SOURCE -DLDB_PTHREAD -DLDB_HAVE_FDATASYNC \
          -DLDB_HAVE_PREAD -fPIC -I$(REF)/include -I$(REF)/src

LIBSRC := $(addprefix src/util/,arena array atomic bloom buffer cache comparator crc32c env \
            hash internal logger options port random rbt slice status strutil \
            thread_pool vector testutil) \
          $(addprefix src/table/,block block_builder filter_block format iterator \
            merger table table_builder two_level_iterator) \
          $(addprefix src/,builder c db_impl db_iter dbformat dumpfile filename \
            log_reader log_writer memtable repair skiplist table_cache version_edit \
            version_set write_batch)
TESTS  := snappy table db corruption simple recovery
LIBOBJ := $(patsubst %,$(OUT)/obj/%.o,$(subst /,__,$(LIBSRC)))
PROGS  := $(addprefix t-,$(TESTS)) build_table dump_blocks
BINS   := $(foreach p,$(PROGS),$(OUT)/$(p).cpu $(OUT)/$(p).gpu) $(OUT)/build_table_batched.gpu

ifneq ($(wildcard $(REF)/src/util/snappy.c),)
all: $(BINS) $(OUT)/libref_bloom.so

$(OUT)/obj/%.o:
	@mkdir -p $(OUT)/obj
	$(CC) $(CFLAGS) -c $(REF)/$(subst __,/,$*).c -o $@

$(OUT)/liblcdb_core.a: $(LIBOBJ)
	ar rcs $@ $^

$(OUT)/refsnappy.o: $(REF)/src/util/snappy.c
	@mkdir -p $(OUT)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/t-%.o: $(REF)/test/t-%.c
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/build_table.o: $(HERE)harness/build_table.c
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/dump_blocks.o: $(HERE)harness/dump_blocks.c
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/build_table_batched.o: $(HERE)harness/build_table_batched.c $(HERE)../include/lcdb_gpu_snappy.h
	$(CC) $(CFLAGS) -I$(HERE)../include -c $< -o $@

# The reference's bloom filter behind a ctypes-callable shim (bloom row pin).
$(OUT)/libref_bloom.so: $(HERE)harness/bloom_ref.c $(OUT)/liblcdb_core.a
	$(CC) $(CFLAGS) -shared $< $(OUT)/liblcdb_core.a -lpthread -o $@

$(OUT)/%.cpu: $(OUT)/%.o $(OUT)/refsnappy.o $(OUT)/liblcdb_core.a
	$(CC) $^ -lpthread -o $@

$(OUT)/%.gpu: $(OUT)/%.o $(OUT)/liblcdb_core.a $(GPULIB)/liblcdb_gpu_snappy.so
	$(CC) $(OUT)/$*.o $(OUT)/liblcdb_core.a -L$(GPULIB) -llcdb_gpu_snappy \
	    -Wl,-rpath,'$$ORIGIN/../../../lcdb_amd' -lpthread -o $@
else
all:
	@echo "reference tree $(REF) absent: using prebuilt $(OUT) binaries if present"
endif

.PHONY: all
.SECONDARY:
