#!/bin/bash
# CI entry point (the reference's .github/workflows/ci.yml runs cargo build/test/clippy and
# the pymoose tests): build every native artefact, run the CPU test suite and the host
# sanitizer builds.  GPU tests run separately on MI355X runners (`make test-gpu`).
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()"
python -m pytest tests -q -m "not gpu" -n "${JOBS:-6}"
scripts/sanitize.sh all
echo "ci: ok"
