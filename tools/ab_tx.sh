#!/bin/bash
# A/B of the transaction-signature kernel (round 2): the committed ecmult
# ("old": radix-16 Booth over 8 Jacobian Q multiples in scratch) against the
# affine, select-read table at window 3 and 4 (DC_SECP_QW).  The variant
# libraries are linked by hand into distributed-chess_amd/build/var/libtx{old,3,4}.so
# (dc_txsig.hip compiled with -DDC_SECP_QW=..., the other objects of `make`).
# Result (MI355X, 262,144 txs): old 6.40 ms, W=3 6.32 ms, W=4 6.56 ms; parity green for all.
set -o pipefail
for v in old 3 4; do
  DCHESS_LIB=$PWD/distributed-chess_amd/build/var/libtx$v.so timeout -k 10 200 python -u -m pytest tests/test_txsig.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/txt_$v.log 2>&1 || { echo "test $v failed"; tail -5 gpurun_out/txt_$v.log; exit 1; }
  tail -1 gpurun_out/txt_$v.log
  DCHESS_LIB=$PWD/distributed-chess_amd/build/var/libtx$v.so timeout -k 10 200 python bench.py --only tx --no-cpu --tx-steps 5 > gpurun_out/txb_$v.json 2> gpurun_out/txb_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/txb_$v.err; exit 2; }
  python -c "import json;d=json.load(open('gpurun_out/txb_$v.json'))['tx_signatures'];print('$v', d['kernel_avg_ms'], d['value'])"
done
# the product library: state-hash parity and leg
timeout -k 10 200 python -u -m pytest tests/test_statehash.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hash_t.log 2>&1 || { tail -5 gpurun_out/hash_t.log; exit 3; }
tail -1 gpurun_out/hash_t.log
timeout -k 10 200 python bench.py --only hash --no-cpu > gpurun_out/hash_b.json 2> gpurun_out/hash_b.err || { tail -5 gpurun_out/hash_b.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/hash_b.json'))['state_hash'];print('hash', d['kernel_avg_ms'], d['value'])"
