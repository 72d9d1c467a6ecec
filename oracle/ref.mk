# oracle/ref.mk -- compile the REFERENCE codec (Grok v5.1.0, libgrok) straight
# from its sources under /root/reference with g++, into oracle/_ref/.
#
# Test infrastructure only (see oracle/grk_oracle.h): the product never links
# or loads anything built here.  Used to
#   * regenerate and check the golden fixtures (oracle/ref_driver.cpp,
#     oracle/make_golden.py, tests/test_ref_pinning.py), and
#   * time the reference CPU path on the GPU box's host cores (bench.py
#     cpu_baseline, kind "reference").
#
# No CMake and no stand-ins: the source list is src/lib/jp2/CMakeLists.txt:
# 37-166 minus the two unit-test mains (util/bench_dwt.cpp,
# util/test_sparse_array.cpp); grk_config.h / grk_config_private.h are made
# from the reference's own *.cmake.in templates by substituting the values
# the reference's CMake would (version 5.1.0 from CMakeLists.txt:35-37, plugin
# name from :26, the header/function probes of :177-191, which all succeed on
# this glibc/x86-64 image).  Compile flags follow src/lib/jp2/CMakeLists.txt
# (C++20, -O3 -DNDEBUG as CMAKE_BUILD_TYPE=Release, -mavx2 -mbmi2 when AVX2 is found, -DSPDLOG_COMPILED_LIB, the
# plugin loader option BUILD_PLUGIN_LOADER=ON -> -DGRK_BUILD_PLUGIN_LOADER).
#
#   make -f oracle/ref.mk          (from the repo root; ~1 min with -j8)
REF ?= /root/reference
SRC := $(REF)/src/lib/jp2
OUT := oracle/_ref
GEN := $(OUT)/gen
CXX ?= g++

CXXFLAGS := -std=c++20 -O3 -DNDEBUG -fPIC -mavx2 -mbmi2 -DSPDLOG_COMPILED_LIB -DGRK_BUILD_PLUGIN_LOADER -w
INC := -I$(GEN) -I$(REF)/src/include -I$(SRC) -I$(SRC)/plugin -I$(SRC)/transform -I$(SRC)/t1 \
       -I$(SRC)/t1/t1_part1 -I$(SRC)/t1/t1_ht -I$(SRC)/t1/t1_ht/coding -I$(SRC)/t1/t1_ht/common \
       -I$(SRC)/t1/t1_ht/others -I$(SRC)/util -I$(SRC)/codestream -I$(SRC)/mct -I$(SRC)/t2

LIBSRCS := util/BufferedStream.cpp util/logger.cpp util/mem_stream.cpp util/grok_malloc.cpp util/util.cpp \
  util/vector.cpp util/CPUArch.cpp util/ChunkBuffer.cpp \
  plugin/minpf_dynamic_library.cpp plugin/minpf_plugin_manager.cpp plugin/plugin_bridge.cpp \
  codestream/BitIO.cpp codestream/j2kprofile.cpp codestream/j2k_dump.cpp codestream/j2k.cpp codestream/jp2.cpp \
  codestream/PacketIter.cpp codestream/TagTree.cpp codestream/Quantizer.cpp codestream/HTParams.cpp \
  mct/invert.cpp mct/mct.cpp t2/T2.cpp t2/RateControl.cpp t2/RateInfo.cpp image.cpp grok.cpp \
  TileBuffer.cpp TileComponent.cpp TileProcessor.cpp \
  transform/Wavelet.cpp transform/sparse_array.cpp transform/dwt.cpp transform/dwt_utils.cpp \
  transform/dwt53.cpp transform/dwt97.cpp \
  t1/T1Decoder.cpp t1/T1Encoder.cpp t1/Tier1.cpp t1/T1Factory.cpp t1/t1_ht/T1HT.cpp \
  t1/t1_ht/coding/ojph_block_decoder.cpp t1/t1_ht/coding/ojph_block_encoder.cpp \
  t1/t1_ht/others/ojph_arch.cpp t1/t1_ht/others/ojph_mem.cpp t1/t1_ht/others/ojph_message.cpp \
  t1/t1_part1/t1.cpp t1/t1_part1/mqc_enc.cpp t1/t1_part1/mqc_dec.cpp t1/t1_part1/T1Part1.cpp
OBJS := $(LIBSRCS:%.cpp=$(OUT)/obj/%.o)

all: $(OUT)/libgrok.so $(OUT)/ref_driver $(OUT)/abi_check $(OUT)/ref_driver_mi355x $(OUT)/tile_driver $(OUT)/tile_driver_mi355x

$(GEN)/grk_config.h: $(SRC)/grk_config.h.cmake.in
	@mkdir -p $(GEN)
	sed -e 's/#cmakedefine GROK_HAVE_STDINT_H.*/#define GROK_HAVE_STDINT_H 1/' \
	    -e 's/@GROK_VERSION_MAJOR@/5/' -e 's/@GROK_VERSION_MINOR@/1/' -e 's/@GROK_VERSION_BUILD@/0/' \
	    -e 's/@GROK_PLUGIN_NAME@/grok_plugin/' -e 's/@AVX2_FOUND@/1/' -e 's/@AVX_FOUND@/1/' \
	    -e 's/@SSE4_1_FOUND@/1/' -e 's/@SSE3_FOUND@/1/' $< > $@

$(GEN)/grk_config_private.h: $(SRC)/grk_config_private.h.cmake.in
	@mkdir -p $(GEN)
	sed -e 's/#cmakedefine GROK_HAVE_INTTYPES_H.*/#define GROK_HAVE_INTTYPES_H 1/' \
	    -e 's/@PACKAGE_VERSION@/5.1.0/' \
	    -e 's|#cmakedefine _LARGEFILE_SOURCE|/* #undef _LARGEFILE_SOURCE */|' \
	    -e 's|#cmakedefine _LARGE_FILES|/* #undef _LARGE_FILES */|' \
	    -e 's|#cmakedefine _FILE_OFFSET_BITS.*|/* #undef _FILE_OFFSET_BITS */|' \
	    -e 's/#cmakedefine GROK_HAVE_FSEEKO.*/#define GROK_HAVE_FSEEKO 1/' \
	    -e 's/#cmakedefine GROK_HAVE_MALLOC_H/#define GROK_HAVE_MALLOC_H/' \
	    -e 's/#cmakedefine GROK_HAVE_ALIGNED_ALLOC/#define GROK_HAVE_ALIGNED_ALLOC/' \
	    -e 's|#cmakedefine GROK_HAVE__ALIGNED_MALLOC|/* #undef GROK_HAVE__ALIGNED_MALLOC */|' \
	    -e 's/#cmakedefine GROK_HAVE_MEMALIGN/#define GROK_HAVE_MEMALIGN/' \
	    -e 's/#cmakedefine GROK_HAVE_POSIX_MEMALIGN/#define GROK_HAVE_POSIX_MEMALIGN/' \
	    -e 's|#cmakedefine GROK_BIG_ENDIAN|/* #undef GROK_BIG_ENDIAN */|' $< > $@

$(OUT)/obj/%.o: $(SRC)/%.cpp $(GEN)/grk_config.h $(GEN)/grk_config_private.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(INC) -c $< -o $@

$(OUT)/libgrok.so: $(OBJS)
	$(CXX) -shared -o $@ $(OBJS) -lpthread -ldl

# fixture driver over the grk_* C API (oracle/ref_driver.cpp)
$(OUT)/ref_driver: oracle/ref_driver.cpp $(OUT)/libgrok.so
	$(CXX) -std=c++17 -O2 -I$(SRC) -I$(GEN) -o $@ oracle/ref_driver.cpp -L$(OUT) -lgrok -Wl,-rpath,'$$ORIGIN' -lpthread

clean:
	rm -rf $(OUT)

.PHONY: all clean

# layout check of include/grk_plugin_abi.h against the reference headers
$(OUT)/abi_check: oracle/abi/abi_check.cpp oracle/abi/abi_ref.cpp oracle/abi/abi_ours.cpp oracle/abi/abi_fields.h include/grk_plugin_abi.h include/grk_api.h $(GEN)/grk_config.h
	$(CXX) -std=c++17 -O0 -w $(INC) -o $@ oracle/abi/abi_check.cpp oracle/abi/abi_ours.cpp oracle/abi/abi_ref.cpp

# the same driver linked against OUR grk_* library (grokimagecompression_amd/
# lib/libgrok.so, include/grk_api.h) instead of the reference's: the grk_* ABI
# drop-in test (tests/test_gpu_grk_api.py)
MILIB := grokimagecompression_amd/lib
$(OUT)/ref_driver_mi355x: oracle/ref_driver.cpp $(MILIB)/libgrok.so $(GEN)/grk_config.h
	$(CXX) -std=c++17 -O2 -I$(SRC) -I$(GEN) -o $@ oracle/ref_driver.cpp -L$(MILIB) -lgrok -Wl,-rpath,'$$ORIGIN/../../$(MILIB)' -lpthread

# the reference's tile-streaming test programs restated (oracle/tile_driver.cpp),
# against the reference's libgrok and against ours (tests/test_gpu_grk_api.py)
$(OUT)/tile_driver: oracle/tile_driver.cpp $(OUT)/libgrok.so
	$(CXX) -std=c++17 -O2 -I$(SRC) -I$(GEN) -o $@ oracle/tile_driver.cpp -L$(OUT) -lgrok -Wl,-rpath,'$$ORIGIN' -lpthread

$(OUT)/tile_driver_mi355x: oracle/tile_driver.cpp $(MILIB)/libgrok.so $(GEN)/grk_config.h
	$(CXX) -std=c++17 -O2 -I$(SRC) -I$(GEN) -o $@ oracle/tile_driver.cpp -L$(MILIB) -lgrok -Wl,-rpath,'$$ORIGIN/../../$(MILIB)' -lpthread
