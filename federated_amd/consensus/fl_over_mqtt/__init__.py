"""Drop-ins for tensorflow2_implementations/FL_over_MQTT/consensus."""
