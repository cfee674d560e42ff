#!/bin/bash
export TMPDIR=/tmp
TAG=r04f ROUNDS=2 LIBS="ws1:ab/ws1.so ws3:ab/ws3.so" bash tools/r04/net_ab.sh || exit 1
echo done
