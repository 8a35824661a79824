"""PDE models of INSR-PDE (advection 1-D, fluid 2-D, elasticity 2-D/3-D) on the `base` API."""
