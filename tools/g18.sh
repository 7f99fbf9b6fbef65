#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
VARIANTS="S3 S3p S3a S3q" DEPTHS="10000 1000" bash tools/gab.sh || exit 1
