"""TEST-ONLY stub."""
