# vep build / test entry points. GPU code targets gfx950 (MI355X) only.
PY      ?= python
HIPCC   ?= hipcc
ARCH    ?= gfx950
SRCS     = $(wildcard csrc/vep/*.cpp)
HIP_SRCS = $(wildcard csrc/vep/*.hip)
TSAN_DIR = build/tsan
ASAN_DIR = build/asan

.PHONY: build test test-gpu bench bench-h265 smoke tsan asan tsan-rpc asan-rpc link-check parse-prof clean

build:                     ## compile the extension in-tree (video_edge_ai_proxy_amd/_vep*.so)
	$(PY) csrc/build.py

test: build                ## CPU test suite
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu: build            ## GPU tests (needs an MI355X)
	$(PY) -m pytest tests -x -q -m gpu

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

bench: build               ## headline benchmark, 1 GPU (torchrun for N > 1)
	$(PY) bench.py

bench-h265: build          ## BASELINE config 5 shape on one GPU: 8 x 4K30 H.265
	$(PY) bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8

# ThreadSanitizer / AddressSanitizer builds of the native stress driver. Sanitizers apply to
# host code only (-Xarch_host); the driver runs the CPU backend, so no GPU is needed.
# Every data-plane source goes in (all csrc/vep/*.cpp host code and every csrc/vep/*.hip kernel
# file, as csrc/build.py does), so the sanitizer binaries link exactly what the module links.
STRESS = csrc/tests/native_stress.cpp csrc/tests/rpc_stress.cpp

$(TSAN_DIR)/native_stress: $(SRCS) $(HIP_SRCS) $(STRESS) $(wildcard csrc/vep/*.h)
	mkdir -p $(TSAN_DIR)
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O1 -g -Xarch_host -fsanitize=thread \
	  $(SRCS) $(STRESS) -x hip $(HIP_SRCS) -o $@ -lpthread

$(ASAN_DIR)/native_stress: $(SRCS) $(HIP_SRCS) $(STRESS) $(wildcard csrc/vep/*.h)
	mkdir -p $(ASAN_DIR)
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O1 -g -Xarch_host -fsanitize=address \
	  -Xarch_host -fno-omit-frame-pointer \
	  $(SRCS) $(STRESS) -x hip $(HIP_SRCS) -o $@ -lpthread

# Cheap link check of the sanitizer target's source set (default CPU suite): the stress driver
# against the data-plane objects csrc/build.py already compiled (no sanitizer instrumentation).
link-check: build
	mkdir -p build/linkcheck
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O0 -c csrc/tests/native_stress.cpp -Icsrc \
	  -o build/linkcheck/native_stress.o
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O0 -c csrc/tests/rpc_stress.cpp -Icsrc \
	  -o build/linkcheck/rpc_stress.o
	$(HIPCC) --offload-arch=$(ARCH) build/linkcheck/native_stress.o build/linkcheck/rpc_stress.o build/obj/vep__*.o \
	  -o build/linkcheck/native_stress -lpthread

tsan: $(TSAN_DIR)/native_stress
	cd /tmp && TSAN_OPTIONS="halt_on_error=1" $(CURDIR)/$(TSAN_DIR)/native_stress

asan: $(ASAN_DIR)/native_stress
	cd /tmp && ASAN_OPTIONS="detect_leaks=1" $(CURDIR)/$(ASAN_DIR)/native_stress

# the native gRPC endpoint's hostile-client stress alone (csrc/tests/rpc_stress.cpp)
tsan-rpc: $(TSAN_DIR)/native_stress
	cd /tmp && TSAN_OPTIONS="halt_on_error=1" $(CURDIR)/$(TSAN_DIR)/native_stress rpc

asan-rpc: $(ASAN_DIR)/native_stress
	cd /tmp && ASAN_OPTIONS="detect_leaks=1" $(CURDIR)/$(ASAN_DIR)/native_stress rpc

# Host parse profile (gprof): the general H.264 decoder over the headline bench's 1080p stream.
build/prof/parse_prof: $(SRCS) $(HIP_SRCS) csrc/tests/parse_prof.cpp $(wildcard csrc/vep/*.h)
	mkdir -p build/prof
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -O2 -g -Xarch_host -pg -Xarch_host -march=x86-64-v3 \
	  -Icsrc $(SRCS) csrc/tests/parse_prof.cpp -x hip $(HIP_SRCS) -o $@ -lpthread

parse-prof: build/prof/parse_prof
	cd /tmp && $(CURDIR)/build/prof/parse_prof 10 && gprof -b -p $(CURDIR)/build/prof/parse_prof /tmp/gmon.out | head -40

clean:
	rm -rf build video_edge_ai_proxy_amd/_vep*.so
