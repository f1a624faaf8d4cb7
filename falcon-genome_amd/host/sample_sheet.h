// Sample sheets of `fcs-genome align -F` (reference SampleSheet,
// /root/reference/include/fcs-genome/SampleSheet.h:19-38,
// src/SampleSheet.cpp:23-215): a CSV whose '#' header names the columns
// (sample_id, fastq1, fastq2, rg, platform_id, library_id, in any order), or a
// folder of <sample>_..._1.fastq.gz / _2.fastq.gz pairs.  Rows of one sample
// become its read groups, in sheet order.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace fcsg {

struct SampleDetails {
  std::string fastqR1, fastqR2, ReadGroup, Platform, LibraryID;
};

typedef std::map<std::string, std::vector<SampleDetails>> SampleSheetMap;

// Parses a sheet file or scans a folder (throws invalidParam / fileNotFound /
// formatError as the reference throws runtime_error).
SampleSheetMap read_sample_sheet(const std::string& path);

}  // namespace fcsg
