# Top-level build: the product library (HIP, gfx950) and the CPU oracle (test infra).
HIPCC ?= /opt/rocm/bin/hipcc
PKG := orb-slam3-noted_amd
CSRC := $(PKG)/csrc
LIBDIR := $(PKG)/lib
HIPFLAGS ?= --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result
SRCS := $(CSRC)/extractor.hip $(CSRC)/matcher.hip $(CSRC)/lba.hip $(CSRC)/pose.hip $(CSRC)/stereo.hip $(CSRC)/mapping.hip $(CSRC)/rectify.hip $(CSRC)/frame.hip $(CSRC)/track.hip
HDRS := $(wildcard $(CSRC)/*.hpp) $(CSRC)/orb_pattern.inc include/slamhot.h

all: $(LIBDIR)/libslamhot.so oracle tests/cpp/host_driver tests/cpp/shim_driver

# C++ host layer (include/slamhot.hpp) driven by tests/test_gpu_cpp_host.py (test infra)
tests/cpp/host_driver: tests/cpp/host_driver.cpp include/slamhot.hpp include/slamhot.h $(LIBDIR)/libslamhot.so
	g++ -O2 -std=c++17 -Wall -Wextra -Iinclude -o $@ $< -L$(LIBDIR) -lslamhot -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

# the drop-in shim bodies (include/slamhot_orbslam3.hpp) on ORB-SLAM3 stand-ins (test infra)
tests/cpp/shim_driver: tests/cpp/shim_driver.cpp tests/cpp/orbslam3_standins.hpp include/slamhot_orbslam3.hpp include/slamhot.hpp include/slamhot.h $(LIBDIR)/libslamhot.so
	g++ -O2 -std=c++17 -Wall -Wextra -Iinclude -o $@ $< -L$(LIBDIR) -lslamhot -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

OBJDIR := build/obj
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS))

# one object per kernel file (parallel make), linked into the one library
$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libslamhot.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(LIBDIR) build oracle/build tests/cpp/host_driver tests/cpp/shim_driver tests/cpp/*_asan

# host-side sanitizer builds (test infrastructure; GPU code is never instrumented): the oracle
# with ASan + UBSan, and the C++ host-layer / shim drivers with ASan + UBSan (tools/sanitize.sh)
SAN := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
sanitize: $(LIBDIR)/libslamhot.so
	cd oracle && g++ $(SAN) -march=x86-64-v3 -ffp-contract=off -fPIC -std=c++17 -shared -o build/liboracle_asan.so *.cpp -lpthread
	g++ $(SAN) -std=c++17 -Iinclude -o tests/cpp/host_driver_asan tests/cpp/host_driver.cpp -L$(LIBDIR) -lslamhot -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'
	g++ $(SAN) -std=c++17 -Iinclude -o tests/cpp/shim_driver_asan tests/cpp/shim_driver.cpp -L$(LIBDIR) -lslamhot -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

# the library's C++ host side under ASan + UBSan (GPU code not instrumented; clang's runtime, which
# the clang++-built drivers load first, so no preload is needed): tools/ab/asan_gpu.sh runs the
# C++ host-layer and shim GPU tests through them
CLANGRT := $(dir $(firstword $(wildcard /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so)))
HIPSAN := --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -ffp-contract=off \
          -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined
sanitize-hip:
	@mkdir -p build/asan $(LIBDIR)/asan
	for f in $(SRCS); do $(HIPCC) $(HIPSAN) -c -o build/asan/$$(basename $$f .hip).o $$f || exit 1; done
	$(HIPCC) $(HIPSAN) -shared -shared-libasan -o $(LIBDIR)/asan/libslamhot.so build/asan/*.o -Wl,-rpath,$(CLANGRT)
	for d in host_driver shim_driver; do /opt/rocm/lib/llvm/bin/clang++ -std=c++17 -O1 -g -fno-omit-frame-pointer \
	  -fsanitize=address,undefined -shared-libasan -Iinclude -o tests/cpp/$${d}_casan tests/cpp/$$d.cpp \
	  -L$(LIBDIR)/asan -lslamhot -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)/asan' -Wl,-rpath,$(CLANGRT) || exit 1; done

.PHONY: all oracle clean sanitize sanitize-hip

# The LBA host planning path of six solver handles at once, each handle's pool growing between
# calls (tests/cpp/plan_stress.cpp), under TSan and under ASan + UBSan (host code instrumented, GPU
# code not; no HIP call is made): tests/test_sanitize_plan.py runs both on the CPU
PLANSAN_SRC := $(CSRC)/lba.hip $(HDRS) tests/cpp/plan_stress.cpp
PLANSAN := --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -ffp-contract=off -DSLAMHOT_PLAN_BENCH
sanitize-plan: tests/cpp/plan_stress_tsan tests/cpp/plan_stress_asan
tests/cpp/plan_stress_tsan: $(PLANSAN_SRC)
	@mkdir -p build/plansan
	$(HIPCC) $(PLANSAN) -Xarch_host -fsanitize=thread -c -o build/plansan/lba_tsan.o $(CSRC)/lba.hip 2>&1 | grep -v "not currently supported for target" || true
	/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=thread -Iinclude -c -o build/plansan/stress_tsan.o tests/cpp/plan_stress.cpp
	$(HIPCC) --hip-link --offload-arch=gfx950 -fsanitize=thread -o $@ build/plansan/stress_tsan.o build/plansan/lba_tsan.o
tests/cpp/plan_stress_asan: $(PLANSAN_SRC)
	@mkdir -p build/plansan
	$(HIPCC) $(PLANSAN) -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -c -o build/plansan/lba_asan.o $(CSRC)/lba.hip 2>&1 | grep -v "not currently supported for target" || true
	/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=address,undefined -Iinclude -c -o build/plansan/stress_asan.o tests/cpp/plan_stress.cpp
	$(HIPCC) --hip-link --offload-arch=gfx950 -fsanitize=address,undefined -o $@ build/plansan/stress_asan.o build/plansan/lba_asan.o
