# Native tools: the C host driver (reference argv, GPU search) and the VALU microbenchmark.
HIPCC ?= /opt/rocm/bin/hipcc
CC    ?= gcc
all: bin/mes_hip bin/mes_seq bin/valu_microbench

bin/mes_hip: tools/mes_main.c include/me.h motionestimation_amd/lib/libme_hip.so
	mkdir -p bin
	$(CC) -O2 -Wall -Iinclude -o $@ tools/mes_main.c -Lmotionestimation_amd/lib -lme_hip \
	    -Wl,-rpath,'$$ORIGIN/../motionestimation_amd/lib' -lm

bin/mes_seq: tools/mes_seq.c include/me.h motionestimation_amd/lib/libme_hip.so
	mkdir -p bin
	$(CC) -O2 -Wall -Iinclude -o $@ tools/mes_seq.c -Lmotionestimation_amd/lib -lme_hip \
	    -Wl,-rpath,'$$ORIGIN/../motionestimation_amd/lib' -lm

bin/valu_microbench: tools/valu_microbench.hip
	mkdir -p bin
	$(HIPCC) --offload-arch=gfx950 -O3 -o $@ $<

.PHONY: all
