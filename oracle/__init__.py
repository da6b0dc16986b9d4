"""TEST INFRASTRUCTURE ONLY: CPU oracle for parity checks (never imported by krr_amd/)."""
