"""plenum_amd — MI355X-native batch Ed25519 request verification for Hyperledger Indy Plenum.

Drop-in for the reference's request-authentication path:
  stp_core.crypto.nacl_wrappers.Verifier / VerifyKey   -> plenum_amd.nacl_wrappers
  plenum.common.verifier.DidVerifier                   -> plenum_amd.verifier
  plenum.server.client_authn.CoreAuthNr (+ authenticate_batch) -> plenum_amd.client_authn
  plenum.server.req_authenticator.ReqAuthenticator (+ authenticate_batch) -> plenum_amd.req_authenticator
The arithmetic runs only in libplenum_verify.so (hand-written gfx950 HIP) through a ctypes C ABI.
"""
__version__ = "0.1.0"
