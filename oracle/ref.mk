# Builds golden-vector drivers against the REFERENCE's own headers, in place
# under /root/reference (read-only; outputs go to oracle/_ref/ only).
# Only pieces that compile from reference + system headers are built here;
# everything needing Boost/Xerces/... is unbuildable in this image.
REF ?= /root/reference
CXX ?= g++
FLAGS := -std=gnu++17 -O2 -ffp-contract=off -DSINGLE_PRECISION -DSPECTRUM_SAMPLES=3 \
         -I$(REF)/include -I$(REF)/src/bsdfs
all: _ref/gl140 _ref/idist
_ref/gl140: ref_drivers/gl140_driver.cpp
	@mkdir -p _ref
	$(CXX) $(FLAGS) $< -o $@
_ref/idist: ref_drivers/idist_driver.cpp
	@mkdir -p _ref
	$(CXX) $(FLAGS) $< -o $@
.PHONY: all
