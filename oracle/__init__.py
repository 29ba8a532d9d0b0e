"""CPU oracle package — TEST INFRASTRUCTURE ONLY (see oracle/salp_oracle.c)."""
