#!/bin/bash
# Regenerates tests/golden/tools_check.txt: the output of tests/native/tools_check.cpp compiled
# against the reference's SiameseTools.h / SiameseSerializers.h (oracle/_ref/tools_check_ref,
# built by oracle/Makefile from /root/reference).
set -e
cd "$(dirname "$0")/../.."
make -C oracle _ref/tools_check_ref
oracle/_ref/tools_check_ref > tests/golden/tools_check.txt
