#!/bin/bash
# Host sanitizer runs that need no GPU: the C restatement under ASan+UBSan
# (every entry point, OpenMP on) and the C ABI runtime's argument-validation and error
# paths under ASan+UBSan and TSan. Logs into profiles/r03/.
set -e
cd "$(dirname "$0")/../.."
mkdir -p profiles/r03
make -s -C oracle SAN=1
make -s -j8 -C ilqr.jl_amd/csrc san SAN=address
make -s -j8 -C ilqr.jl_amd/csrc san SAN=thread
{
  echo "== oracle/lib/san_driver (ASan + UBSan, leak check on)"; ./oracle/lib/san_driver
  echo "== ilqr.jl_amd/lib/san_address/abi_driver (ASan + UBSan, leak check on)"; ./ilqr.jl_amd/lib/san_address/abi_driver
  echo "== ilqr.jl_amd/lib/san_thread/abi_driver (TSan)"; ./ilqr.jl_amd/lib/san_thread/abi_driver
} 2>&1 | tee profiles/r03/san_cpu.log
