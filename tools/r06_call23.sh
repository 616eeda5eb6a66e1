#!/bin/bash
# round 6: the randomized lean / quiesce / encode-toggle test
cd "$GRAFT_REPO_ROOT"
tools/gpu_tests.sh r06_rand 900 tests/test_gpu_lean.py || exit 1
