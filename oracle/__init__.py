"""CPU oracle for the SVGD hot path -- TEST INFRASTRUCTURE ONLY (see svgd_oracle.py)."""
