set -e
TAG=r02an VAR=inl bash tools/ab_lib.sh
TAG=r02an VAR=inl2 CFGS=c3 bash tools/ab_lib.sh
