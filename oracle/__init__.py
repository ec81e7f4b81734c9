"""TEST INFRASTRUCTURE ONLY: CPU oracle (fp64 C restatement) used as the checker."""
