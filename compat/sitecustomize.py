"""Auto-attach hooks that a SageMaker training container would (compat layer, training jobs only)."""
import os

if os.environ.get("MI355X_DP_DEBUGGER"):
    try:
        from mi355x_dp.trace.debugger import install_from_env
        install_from_env()
    except Exception as e:  # never break user code because of observability
        print(f"[mi355x_dp.debugger] not attached: {e!r}", flush=True)
