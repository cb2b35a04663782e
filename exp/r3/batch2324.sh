#!/bin/bash
# batches 23 and 24 in one call
bash exp/r3/batch23.sh && bash exp/r3/batch24.sh
