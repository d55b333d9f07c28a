"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see griffin_ref.py)."""
