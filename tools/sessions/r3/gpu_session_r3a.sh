set -o pipefail
export TMPDIR=/tmp
STAGES="test bench prof pmc fidepmc" bash tools/gpu_round.sh || exit $?
TAG=soa_r2 DCHESS_LIB=$PWD/distributed-chess_amd/build/var/lib_soa_r2.so timeout -k 10 120 python -u tools/c2c_diag.py 3 > gpurun_out/c2c_diag_soa_r2.jsonl 2>&1 || exit 9
