"""TEST-ONLY: expose the oracle's base58 restatement under the package name the reference imports."""
import os, sys
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))
from oracle.base58_ref import *  # noqa
from oracle.base58_ref import b58decode, b58encode, b58decode_int, b58encode_int, BITCOIN_ALPHABET, alphabet  # noqa
