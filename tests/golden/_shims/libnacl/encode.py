"""TEST-ONLY: libnacl.encode helpers."""
import base64, binascii
def hex_encode(data): return binascii.hexlify(data)
def hex_decode(data): return binascii.unhexlify(data)
def base16_encode(data): return base64.b16encode(data)
def base16_decode(data): return base64.b16decode(data)
def base32_encode(data): return base64.b32encode(data)
def base32_decode(data): return base64.b32decode(data)
def base64_encode(data): return base64.b64encode(data)
def base64_decode(data): return base64.b64decode(data)
