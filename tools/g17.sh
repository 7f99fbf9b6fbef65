#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
VARIANTS="A0 A4 S3 S4 F1n" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
