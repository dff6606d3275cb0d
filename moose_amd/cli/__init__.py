"""Command-line tools (reference ``moose/src/bin``): ``elk`` compiler, ``dasher`` local
simulator, ``comet``/``cometctl`` worker + client, ``rudolph`` filesystem-choreography
worker, ``vixen`` per-party runner of compiled graphs."""
