# Builds the HIP C-ABI library in-tree (travels to the GPU box with the repo).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := hyperopt_amd/csrc
SRCS := $(CSRC)/tpe_fit.hip $(CSRC)/tpe_parzen.hip $(CSRC)/tpe_score.hip $(CSRC)/tpe_table.hip $(CSRC)/tpe_history.hip $(CSRC)/tpe_sorted.hip $(CSRC)/tpe_prior.hip $(CSRC)/tpe_dist.hip $(CSRC)/tpe_util.hip $(CSRC)/tpe_ops.hip
OBJS := $(SRCS:.hip=.o)
LIB := hyperopt_amd/libtpe_hip.so
# -ffp-contract=off: no implicit FMA fusion, so expressions written to
# follow numpy's operation order (linspace ramps, normal_cdf, erf-pair sums)
# round exactly as numpy does; hot loops spell their FMAs out (fmaf).
# EXTRA: diagnostic defines for A/B variant builds (tools/mkvariant.sh); empty in the product
EXTRA ?=
FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -ffp-contract=off $(EXTRA)

all: $(LIB)

$(CSRC)/%.o: $(CSRC)/%.hip $(CSRC)/tpe_common.hpp $(CSRC)/tpe_sample.hpp include/tpe_hip.h
	$(HIPCC) $(FLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -f $(OBJS) $(LIB)

.PHONY: all clean
