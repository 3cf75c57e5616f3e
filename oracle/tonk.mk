# Tonk's own unit_tests (tests/TonkUnitTest.cpp: sender bandwidth control, 100 full-duplex lossy
# transfers under the Mau simulator with memcmp checks, ...) built straight from the reference
# sources under REF, twice:
#   _ref/tonk/unit_tests_ref : with the reference Siamese codec (gf256/siamese/Siamese*.cpp)
#   _ref/tonk/unit_tests_amd : Tonk's sources compiled against OUR headers -- include/siamese.h,
#                              include/SiameseTools.h, include/SiameseSerializers.h (SURVEY
#                              s8(b): the header-compatible helpers TonkineseTools.h:61-62 pulls
#                              in) -- and linked with libtonk_amd.so instead of the reference codec
#                              and its SiameseTools.cpp (the clocks come from the library)
#   _ref/tonk/unit_tests_amd_lz : and the compressor too: PacketCompression.cpp replaced by
#                                 integration/tonk/PacketCompressionAmd.cpp
# Nothing is copied into the repository; outputs go to oracle/_ref/ (git-ignored).
#
#   make -C oracle -f tonk.mk -j8
REF      ?= /root/reference
OUT      := _ref/tonk
CXX      ?= g++
CC       ?= gcc
ARCH     := -march=x86-64-v3
# compile definitions as the reference CMakeLists gives them: tonk_static (CMakeLists.txt:214)
# for the library, none for the Mau simulator and the test sources
LIB_DEFS := -DSIAMESE_BUILDING=1 -DTONK_BUILDING=1 -DTONK_DISABLE_SHIM=1
INCS     := -I$(REF) -I$(REF)/thirdparty
CXXFLAGS := -std=c++11 -O2 $(ARCH) -w $(INCS)
# our headers first for every quoted include; -I- also stops the includer's own directory (the
# reference tree) from being searched first, so "siamese.h", "SiameseTools.h" and
# "SiameseSerializers.h" resolve to ../include
AMD_CXXFLAGS := -std=c++11 -O2 $(ARCH) -w -I../include -I- $(INCS)
CFLAGS   := -O2 $(ARCH) -w $(INCS)

TONK_CPP := tonk.cpp tonk_file_transfer.cpp MappedFile.cpp TonkineseBandwidth.cpp TonkineseConnection.cpp \
            SimpleCipher.cpp StrikeRegister.cpp PacketCompression.cpp TonkineseFirewall.cpp TonkineseFlood.cpp \
            TonkineseIncoming.cpp TonkineseMaps.cpp TonkineseOutgoing.cpp TonkineseProtocol.cpp \
            TonkineseSession.cpp TonkineseTools.cpp TonkineseUDP.cpp TonkineseNAT.cpp WLANOptimizer.cpp \
            TimeSync.cpp SiameseTools.cpp Logger.cpp PacketAllocator.cpp cymric.cpp TonkCppSDK.cpp
TEST_CPP := tests/mau/mau.cpp tests/mau/MauProxy.cpp tests/mau/MauTools.cpp \
            tests/TonkUnitTest.cpp tests/BandwidthControlTest.cpp tests/TonkTestTools.cpp
CODEC_CPP := gf256.cpp siamese.cpp SiameseCommon.cpp SiameseDecoder.cpp SiameseEncoder.cpp
TONK_C   := thirdparty/blake2b-ref.c thirdparty/chacha.c thirdparty/chacha_blocks_ref.c thirdparty/t1ha.c \
            $(addprefix thirdparty/zstd/,entropy_common.c error_private.c fse_compress.c fse_decompress.c \
              huf_compress.c huf_decompress.c xxhash.c zstd_common.c zstd_compress.c zstd_decompress.c \
              zstd_double_fast.c zstd_fast.c zstd_lazy.c zstd_ldm.c zstd_opt.c)

obj = $(OUT)/obj/$(subst /,_,$(1)).o
aobj = $(OUT)/obj_amd/$(subst /,_,$(1)).o
TONK_OBJS  := $(foreach f,$(TONK_CPP) $(TONK_C) $(TEST_CPP),$(call obj,$(f)))
CODEC_OBJS := $(foreach f,$(CODEC_CPP),$(call obj,$(f)))
# the drop-in build: every Tonk C++ source against our headers; the reference's SiameseTools.cpp
# is not linked (libtonk_amd.so exports siamese::GetTimeUsec / GetTimeMsec)
AMD_CPP    := $(filter-out SiameseTools.cpp,$(TONK_CPP))
AMD_OBJS   := $(foreach f,$(AMD_CPP) $(TEST_CPP),$(call aobj,$(f))) $(foreach f,$(TONK_C),$(call obj,$(f)))

all: $(OUT)/unit_tests_ref $(OUT)/unit_tests_amd $(OUT)/unit_tests_amd_lz

define compile_rule
$(call obj,$(1)): $(REF)/$(1)
	@mkdir -p $(OUT)/obj
	$(if $(filter %.c,$(1)),$(CC) $(CFLAGS),$(CXX) $(CXXFLAGS)) $(2) -c -o $$@ $$<
endef
$(foreach f,$(TONK_CPP) $(TONK_C) $(CODEC_CPP),$(eval $(call compile_rule,$(f),$(LIB_DEFS))))
$(foreach f,$(TEST_CPP),$(eval $(call compile_rule,$(f),)))

AMD_HDRS := ../include/siamese.h ../include/SiameseTools.h ../include/SiameseSerializers.h
define amd_rule
$(call aobj,$(1)): $(REF)/$(1) $(AMD_HDRS)
	@mkdir -p $(OUT)/obj_amd
	$(CXX) $(AMD_CXXFLAGS) -I$(dir $(REF)/$(1)) $(2) -c -o $$@ $$<
endef
$(foreach f,$(AMD_CPP),$(eval $(call amd_rule,$(f),$(LIB_DEFS))))
$(foreach f,$(TEST_CPP),$(eval $(call amd_rule,$(f),)))

$(OUT)/unit_tests_ref: $(TONK_OBJS) $(CODEC_OBJS)
	$(CXX) -o $@ $^ -lpthread -ldl

$(OUT)/unit_tests_amd: $(AMD_OBJS) ../tonk_amd/libtonk_amd.so
	$(CXX) -o $@ $(AMD_OBJS) -L../tonk_amd -ltonk_amd -Wl,-rpath,'$$ORIGIN/../../../tonk_amd' -lpthread -ldl

LZ_SHIM := $(OUT)/obj/PacketCompressionAmd.o
$(LZ_SHIM): ../integration/tonk/PacketCompressionAmd.cpp ../include/tonk_compress.h $(AMD_HDRS)
	@mkdir -p $(OUT)/obj
	$(CXX) $(AMD_CXXFLAGS) $(LIB_DEFS) -c -o $@ $<

$(OUT)/unit_tests_amd_lz: $(filter-out $(call aobj,PacketCompression.cpp),$(AMD_OBJS)) $(LZ_SHIM) ../tonk_amd/libtonk_amd.so
	$(CXX) -o $@ $(filter-out $(call aobj,PacketCompression.cpp),$(AMD_OBJS)) $(LZ_SHIM) -L../tonk_amd -ltonk_amd \
	    -Wl,-rpath,'$$ORIGIN/../../../tonk_amd' -lpthread -ldl

.PHONY: all
