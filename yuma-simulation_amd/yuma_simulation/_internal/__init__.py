"""Internal implementation of yuma_simulation on the MI355X engine.

As in the reference, public imports go through the versioned ``v1`` package.
"""
