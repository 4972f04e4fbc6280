"""Drop-ins for tensorflow2_implementations/FL_radar_dataset/consensus (ring rule for N < 2)."""
