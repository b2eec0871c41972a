"""TEST INFRASTRUCTURE ONLY — the CPU oracle (see honu_oracle.h)."""
