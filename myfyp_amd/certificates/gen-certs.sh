#!/bin/bash
# Generate a throw-away CA + server/client certificates for the gRPC transport's mutual TLS
# (SAN 127.0.0.1 / ::1 / localhost). Parity: p2pfl/certificates/gen-certs.sh.
set -euo pipefail
cd "$(dirname "$0")"
DAYS=${DAYS:-365}
openssl req -x509 -newkey rsa:2048 -nodes -days "$DAYS" -keyout ca.key -out ca.crt -subj "/CN=myfyp-ca" 2>/dev/null
cat > san.cnf <<CNF
subjectAltName = IP:127.0.0.1, IP:::1, DNS:localhost
CNF
for who in server client; do
  openssl req -newkey rsa:2048 -nodes -keyout "$who.key" -out "$who.csr" -subj "/CN=myfyp-$who" 2>/dev/null
  openssl x509 -req -in "$who.csr" -CA ca.crt -CAkey ca.key -CAcreateserial -out "$who.crt" -days "$DAYS" -extfile san.cnf 2>/dev/null
  rm -f "$who.csr"
done
rm -f san.cnf ca.srl
echo "certificates written to $(pwd)"
