# oracle/ref.mk -- TEST INFRASTRUCTURE ONLY.
#
# Builds the reference CPU KLT library (FatimaSohailll/KLT-Feature-Tracker-
# Acceleration-GPUs, src/V3 `make cpu` path) straight from the sources where
# they lie under /root/reference.  Nothing is copied into the repository; all
# outputs go to oracle/_ref/ (git-ignored, but it travels to the GPU box with
# gpurun so the box can time the real reference as the CPU baseline).
#
# Flags follow src/V3/Makefile:8-9 (gcc -DNDEBUG -O3) minus -pg, plus -fPIC so
# the same objects can form a shared library for ctypes.  The reference
# Makefile links -lcudart -lcuda into the CPU target for no reason
# (src/V3/Makefile:36,58); we link -lm only.
#
#   make -f oracle/ref.mk            # libklt_ref.so + example3_ref + example3_v1
#
REF      ?= /root/reference
V3       := $(REF)/src/V3
V1       := $(REF)/src/V1
OUT      := $(dir $(lastword $(MAKEFILE_LIST)))_ref
CC       := gcc
CFLAGS   := -DNDEBUG -O3 -fPIC -w
LIBSRC   := convolve.c error.c pnmio.c pyramid.c selectGoodFeatures.c \
            storeFeatures.c trackFeatures.c klt.c klt_util.c writeFeatures.c

V3OBJ    := $(addprefix $(OUT)/v3/,$(LIBSRC:.c=.o))
V1OBJ    := $(addprefix $(OUT)/v1/,$(LIBSRC:.c=.o))

all: $(OUT)/libklt_ref.so $(OUT)/example3_ref $(OUT)/example3_v1

$(OUT)/v3/%.o: $(V3)/%.c
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -I$(V3) -c $< -o $@

$(OUT)/v1/%.o: $(V1)/%.c
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -I$(V1) -c $< -o $@

$(OUT)/libklt_ref.so: $(V3OBJ)
	$(CC) -shared -o $@ $^ -lm

# src/V3/example3.c: `example3_ref <dataset> <nFeatures> <nFrames>`, reads
# ../../data/<dataset>/img%d.pgm relative to its working directory.
$(OUT)/example3_ref: $(V3)/example3.c $(V3OBJ)
	$(CC) $(CFLAGS) -I$(V3) -o $@ $^ -lm

# src/V1/example3.c: fixed images_provided/img0.., 150 features, 10 frames.
$(OUT)/example3_v1: $(V1)/example3.c $(V1OBJ)
	$(CC) $(CFLAGS) -I$(V1) -o $@ $^ -lm

# The reference's own harness relinked against OUR drop-in library (the
# integration proof in INTEGRATION.md): same example3.c object, different lib.
AMDLIB   ?= $(abspath $(OUT)/../../klt-feature-tracker-acceleration-gpus_amd/lib)
$(OUT)/example3_amd: $(V3)/example3.c
	$(CC) -DNDEBUG -O3 -w -I$(V3) -o $@ $< -L$(AMDLIB) -lklt_amd -Wl,-rpath,'$$ORIGIN/../../klt-feature-tracker-acceleration-gpus_amd/lib' -lm

.PHONY: all
