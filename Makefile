# Top-level build: libdct3d.so (HIP kernels + C-ABI runtime, gfx950) and libdct3dcodec.so + the
# dct3d_codec CLI (the reference-compatible C codec host: encode()/decode(), cube pack/unpack,
# diagonal slices, Exp-Golomb, zlib).  Objects go to build/, libraries into the package (git-ignored,
# they travel to the GPU box with the gpurun snapshot).
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
PKG     := 3ddctvideoencoding_amd
CSRC    := $(PKG)/csrc
LIBDIR  := $(PKG)/lib
OBJ     := build/obj
# -ffp-contract=off: the certification bounds (dct3d_plan.cpp) are derived for exactly the written
# operation sequence; no FMA contraction behind its back.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Iinclude $(EXTRA_HIPFLAGS)
CFLAGS   := -O2 -fPIC -Wall -Wextra -Wno-unused-parameter -Iinclude -std=c11 -D_GNU_SOURCE

DEV_SRCS  := $(CSRC)/dct3d_kernels.hip $(CSRC)/dct3d_kernels_f.hip $(CSRC)/dct3d_eg.hip
DIAG_SRCS := $(CSRC)/dct3d_diag.hip
HOST_SRCS := $(CSRC)/dct3d_plan.cpp $(CSRC)/dct3d_runtime.cpp
HDRS      := $(wildcard $(CSRC)/*.h) include/dct3d.h include/dct3d_diag.h
CODEC_SRCS := $(wildcard $(CSRC)/host/*.c)
CODEC_LIB_SRCS := $(filter-out $(CSRC)/host/main.c,$(CODEC_SRCS))

LIB      := $(LIBDIR)/libdct3d.so
DIAGLIB  := $(LIBDIR)/libdct3d_diag.so
CODECLIB := $(LIBDIR)/libdct3dcodec.so
CLI      := $(LIBDIR)/dct3d_codec

all: $(LIB) $(DIAGLIB) $(if $(CODEC_LIB_SRCS),$(CODECLIB) $(CLI))

$(OBJ)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -x hip --offload-arch=$(ARCH) -c $< -o $@

$(LIB): $(patsubst $(CSRC)/%.hip,$(OBJ)/%.o,$(DEV_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJ)/%.o,$(HOST_SRCS))
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

# measurement / test support (include/dct3d_diag.h): never linked into the product library
$(DIAGLIB): $(patsubst $(CSRC)/%.hip,$(OBJ)/%.o,$(DIAG_SRCS)) $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(patsubst $(CSRC)/%.hip,$(OBJ)/%.o,$(DIAG_SRCS)) -L$(LIBDIR) -ldct3d -Wl,-rpath,'$$ORIGIN'

$(CODECLIB): $(CODEC_LIB_SRCS) $(LIB) $(wildcard include/*.h)
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -shared -o $@ $(CODEC_LIB_SRCS) -L$(LIBDIR) -ldct3d -Wl,-rpath,'$$ORIGIN' -lz -lm -lpthread

$(CLI): $(CSRC)/host/main.c $(CODECLIB)
	$(CC) $(CFLAGS) -o $@ $< -L$(LIBDIR) -ldct3dcodec -ldct3d -Wl,-rpath,'$$ORIGIN' -lz -lm -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIBDIR)

.PHONY: all clean oracle
