"""bcos_gpu -- MI355X-native batch-verification engine for FISCO-BCOS's tx-admission and
block-check hot path (host-side mirror of the reference's bcos-crypto interfaces over the
libbcosgpu.so C ABI; see include/bcos_gpu.h and DESIGN.md)."""
from . import _lib
from ._lib import (BcosGpuError, check, clear_keys, ensure_device, header_symbols, key_cache_info, lib,
                   register_keys, set_tx_kernel_policy)
from .crypto import (SM3, CryptoSuite, Hash, InvalidSignature, Keccak256, Merkle, SM2Crypto,
                     Secp256k1Crypto, calculate_merkle_proof_root, pack_messages, right160,
                     secp256k1_suite, sm_suite)
from . import tars
from .tx import (LogEntry, Transaction, TransactionData, TransactionReceipt, TransactionReceiptData,
                 calculate_receipt_root, calculate_roots_batch, calculate_transaction_root, verify_packed,
                 verify_transactions)

__all__ = [n for n in dir() if not n.startswith("_")]
