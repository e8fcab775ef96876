"""Public interface of the yuma_simulation package, API version 1."""
