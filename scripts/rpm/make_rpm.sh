#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/../.."
V=0.1.0
mkdir -p ~/rpmbuild/{SOURCES,SPECS}
git archive --prefix="dynolog-amd-$V/" -o ~/rpmbuild/SOURCES/dynolog-amd-$V.tar.gz HEAD
cp scripts/rpm/dynolog.spec ~/rpmbuild/SPECS/
rpmbuild -ba ~/rpmbuild/SPECS/dynolog.spec
