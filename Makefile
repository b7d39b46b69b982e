# Builds the MI355X (gfx950) AD-Census library and the CPU oracle.
#   make            -> tea_stereo_matching_amd/lib/libtsm_adcensus.so + oracle/build/liboracle_adcensus.so
#   make -j16 lib   -> library only
# -ffp-contract=off: hipcc contracts a*b+c into FMA by default, which would break
# bit-exactness with the reference's uncontracted float expressions.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
SRC      := tea_stereo_matching_amd/csrc
OBJ      := build/obj
LIBDIR   := tea_stereo_matching_amd/lib
LIB      := $(LIBDIR)/libtsm_adcensus.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++20 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result -Wno-unused-value -Iinclude
HIP_SRCS := k_cost k_aggregate k_scanline k_refine k_stereo_ops
CPP_SRCS := engine stereo_ops
OBJS     := $(addprefix $(OBJ)/,$(addsuffix .o,$(HIP_SRCS) $(CPP_SRCS)))
HDRS     := $(SRC)/copy_pool.h $(SRC)/tsm_device.h $(SRC)/tsm_launch.h include/tsm_adcensus.h include/stereo.h include/tsm_stereo_ops.h

all: lib oracle probe

# HBM calibration kernels for bench.py (measurement tooling, not the product)
PROBE    := tools/lib/libtsm_hbm_probe.so
probe: $(PROBE)
$(PROBE): tools/micro/hbm_probe.hip
	@mkdir -p tools/lib
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++20 -fPIC -Wno-unused-result -shared -o $@ $<

lib: $(LIB)

$(OBJ)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

# experimental variants for on-GPU A/B timing, built from a copy of the sources with a
# patch applied (the product sources carry no probes):
#   make exp X=name PATCH=tools/probes/name.patch [DEFS=...]
EXP = build/exp/$(X)
exp:
	@test -n "$(X)" || { echo 'make exp: X=<name> required'; exit 1; }
	@test -z "$(PATCH)" || test -f "$(PATCH)" || { echo 'make exp: PATCH=$(PATCH) not found'; exit 1; }
	rm -rf $(EXP)/tea_stereo_matching_amd $(EXP)/include $(EXP)/obj
	mkdir -p $(EXP)/tea_stereo_matching_amd $(EXP)/obj
	cp -r include $(EXP)/include
	cp -r $(SRC) $(EXP)/tea_stereo_matching_amd/csrc
	if [ -n "$(PATCH)" ]; then patch -p1 -d $(EXP) < $(PATCH) || exit 1; fi
	for f in $(HIP_SRCS); do $(HIPCC) $(HIPFLAGS) $(DEFS) -c $(EXP)/$(SRC)/$$f.hip -o $(EXP)/obj/$$f.o || exit 1; done
	for f in $(CPP_SRCS); do $(HIPCC) $(HIPFLAGS) $(DEFS) -c $(EXP)/$(SRC)/$$f.cpp -o $(EXP)/obj/$$f.o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(EXP)/libtsm_adcensus.so $(EXP)/obj/*.o

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIBDIR)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean exp probe
