# Build / test entry points (reference: Makefile + .travis.yml — build the
# cmd/ binaries, run the test suite).
PY ?= python

.PHONY: build test test-gpu lint sanitize bench smoke simul clean

build:            ## compile every HIP translation unit for gfx950 into drynx_amd/native/libdrynx_native.so
	$(PY) -m drynx_amd.native.build

test: build       ## CPU suite (host path of the same kernels, gloo multi-rank)
	$(PY) -m pytest tests -m "not gpu" -q -n 4

lint:             ## stdlib source lint (syntax, unused imports, whitespace, line length, no CUDA spellings)
	$(PY) tools/lint.py

test-gpu: build   ## on an MI355X
	$(PY) -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread

sanitize:         ## CPU suite against the host-ASan/UBSan build of the native library
	$(PY) -m drynx_amd.native.build --sanitize
	LD_PRELOAD=$$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so) ASAN_OPTIONS=detect_leaks=0 \
	  DRYNX_NATIVE_LIB=build/libdrynx_native_asan.so $(PY) -m pytest tests -m "not gpu" -q -p no:cacheprovider

bench: build      ## headline benchmark, 1 GPU (N GPUs: torch.distributed.run ... bench.py --gpus N)
	$(PY) bench.py --steps 3 --warmup 1

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

simul: build      ## onet-style runfile simulation with named-timer CSV
	$(PY) -m drynx_amd.simul.simul drynx_amd/simul/runfiles/drynx.toml --csv timers.csv

clean:
	rm -rf build drynx_amd/native/libdrynx_native.so drynx_amd/native/libdrynx_native.so.stamp
