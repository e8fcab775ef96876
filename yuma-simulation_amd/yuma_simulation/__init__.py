"""Public interface of the yuma_simulation package (MI355X-native engine)."""
